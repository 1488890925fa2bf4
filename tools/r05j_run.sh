#!/bin/bash
# round 5 final build, multi-GPU evidence on one GPU: every rank's share of the 8 / 4 / 2-GPU layouts at full size
# (verified), RCCL rehearsals of N = 8 and N = 2 with the verified bench line, the merge bench, heavy / symbolic stamps
set -u
T=r05j
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
tools/gpu_steps.sh $T share:8:22 share:4:21 share:2:21 dist:8:19 dist:2:18 || exit $?
timeout -k 10 300 python3 -u tools/bench_merge.py --scale 20 --reps 3 > $OUT/merge_s20.log 2>&1 || { tail -5 $OUT/merge_s20.log; exit 30; }
tail -1 $OUT/merge_s20.log | cut -c1-300
timeout -k 10 300 python3 -u tools/diag_stamps.py 20 > $OUT/diag_stamps_s20.txt 2>&1 || { tail -5 $OUT/diag_stamps_s20.txt; exit 31; }
grep k_sym_part $OUT/diag_stamps_s20.txt
timeout -k 10 300 python3 -u tools/diag_known.py > $OUT/diag_known.txt 2>&1 || { tail -5 $OUT/diag_known.txt; exit 32; }
head -14 $OUT/diag_known.txt
