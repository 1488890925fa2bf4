#!/bin/bash
# round-5 evidence call: GPU suite, N = 1 bench, s22 2x2x2 rank shares (verified), N = 8 RCCL rehearsal at s19,
# k_sym_part / heavy stamps, part-table A/B
set -u
tools/gpu_steps.sh r05a tests bench share:8:22 dist:8:19 || exit $?
OUT=gpurun_out/r05a
timeout -k 10 300 python3 -u tools/diag_stamps.py 20 > "$OUT/diag_stamps_s20.txt" 2>&1 || exit 30
tail -4 "$OUT/diag_stamps_s20.txt"
for s in 20 21; do
  CBG_PART_TABLE=0 timeout -k 10 300 python3 -u bench.py --no-cpu --steps 5 --scale $s > "$OUT/noptab_s$s.log" 2>&1 || exit 31
  tail -1 "$OUT/noptab_s$s.log" | cut -c1-300
done
