#!/bin/bash
# Rehearse bench.py's distributed path on a one-GPU box, every rank on cuda:0.
#   BACKEND=rccl-net (default): libcbgpu's own RCCL grid, each rank its own RCCL "node" (NCCL_HOSTID) so RCCL's
#                               socket transport carries the bytes (the production RCCL calls, slow wire)
#   BACKEND=gloo:               the host-staged caller transport
# usage: tools/gpu_dist_rehearsal.sh N scale [extra bench args]   (env passes through, e.g. CBG_FIBER_PIPE=0)
set -u
N=${1:-2}; SCALE=${2:-14}; shift 2 || true
TAG=${TAG:-dist}
mkdir -p gpurun_out
CBG_DIST_BACKEND=${BACKEND:-rccl-net} timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port ${PORT:-29650} bench.py --gpus $N --steps 2 --warmup 1 --scale $SCALE "$@" \
  > gpurun_out/${TAG}_$N.log 2>&1
rc=$?; echo "rehearsal N=$N rc=$rc"; grep '^{' gpurun_out/${TAG}_$N.log | tail -1 | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config']['parallelism'], 'ms/step', round(d['ms_per_step'],2), d.get('rank0_phases_per_step'))" || tail -5 gpurun_out/${TAG}_$N.log
exit $rc
