#!/bin/bash
# u16/f32 per-direction fiber narrowing: distributed GPU tests + 2-rank rehearsal (fiber bytes)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03af; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
TAG=r03af/n16gap bash tools/gpu_dist_rehearsal.sh 2 16 --no-cpu
TAG=r03af/n16gapoff CBG_FIBER_GAPS=0 PORT=29651 bash tools/gpu_dist_rehearsal.sh 2 16 --no-cpu
