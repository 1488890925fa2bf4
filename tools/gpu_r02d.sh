#!/bin/bash
set -u
mkdir -p gpurun_out/r02d
timeout -k 10 300 python3 -u tools/diag_stamps.py 20 > gpurun_out/r02d/stamps.log 2>&1; echo "stamps rc=$?"; cat gpurun_out/r02d/stamps.log | tail -25
for N in 2 4 8; do
  bash tools/gpu_dist_rehearsal.sh $N 16 || exit $?
done
