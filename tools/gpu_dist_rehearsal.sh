#!/bin/bash
# Rehearse bench.py's distributed path on a one-GPU box: gloo ranks sharing cuda:0 (the RCCL path
# needs one GPU per rank).  usage: tools/gpu_dist_rehearsal.sh N scale
set -u
N=${1:-2}; SCALE=${2:-14}
mkdir -p gpurun_out
CBG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29650 bench.py --gpus $N --steps 2 --warmup 1 --scale $SCALE \
  > gpurun_out/dist_rehearsal_$N.log 2>&1
rc=$?; echo "rehearsal N=$N rc=$rc"; tail -3 gpurun_out/dist_rehearsal_$N.log; exit $rc
