#!/bin/bash
# A/B of the symbolic part table (CBG_PART_TABLE) at s20 / s21, the heavy-kernel stamps (tools/diag_known.py) and the
# local-product GPU tests, in one gpurun call (exit 10 + step on failure).
set -u
OUT=gpurun_out/${1:-r05n}
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in 20 21; do
  CBG_PART_TABLE=0 timeout -k 10 300 python3 -u bench.py --no-cpu --steps 5 --scale $s > "$OUT/noptab_s$s.log" 2>&1 || exit 11
  timeout -k 10 300 python3 -u bench.py --no-cpu --steps 5 --scale $s > "$OUT/ptab_s$s.log" 2>&1 || exit 12
done
timeout -k 10 300 python3 -u tools/diag_known.py > "$OUT/diag_known.txt" 2>&1 || exit 13
tools/gpu_steps.sh "${1:-r05n}" tests:spgemm
