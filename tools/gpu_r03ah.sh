#!/bin/bash
# one-GPU RCCL rehearsal of the mandated layouts with the round-3 fiber formats (u16 values, 16-bit row gaps)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03ah
TAG=r03ah/n2s18 bash tools/gpu_dist_rehearsal.sh 2 18 --no-cpu
TAG=r03ah/n2s18off CBG_FIBER_GAPS=0 CBG_FIBER_NARROW=0 PORT=29652 bash tools/gpu_dist_rehearsal.sh 2 18 --no-cpu
TAG=r03ah/n8s19 PORT=29653 bash tools/gpu_dist_rehearsal.sh 8 19 --no-cpu
