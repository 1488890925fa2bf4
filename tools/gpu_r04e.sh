#!/bin/bash
# r04e: rank shares (2x2x2 s22 rank 0; 1x1x2 s21 both ranks, with the workspace release before the merge), merge
# (packed window scan vs round 3), symbolic variants (8 waves, 2^19-row parts), one-GPU RCCL rehearsals.
set -u
OUT=gpurun_out/r04e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_merge.py --scale 20 --reps 3 > $OUT/merge.log 2>&1 || { tail -5 $OUT/merge.log; exit 4; }

tail -qn1 $OUT/merge.log | cut -c1-700
timeout -k 10 600 python -u bench.py --rank-share 0 --gpus-virtual 8 --scale 22 > $OUT/rank_share_s22.jsonl 2> $OUT/rank_share.err || { tail -5 $OUT/rank_share.err; exit 13; }
timeout -k 10 600 python -u bench.py --rank-share all --gpus-virtual 2 --scale 21 > $OUT/rank_share_s21_n2.jsonl 2> $OUT/rank_share2.err || { tail -5 $OUT/rank_share2.err; exit 13; }
timeout -k 10 600 python -u bench.py --rank-share 0 --gpus-virtual 4 --scale 21 > $OUT/rank_share_s21_n4.jsonl 2> $OUT/rank_share4.err || { tail -5 $OUT/rank_share4.err; exit 13; }
cut -c1-600 $OUT/rank_share_*.jsonl
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 --warmup 2 > $OUT/s20_main.log 2>&1 || exit 5
timeout -k 10 300 python3 -u tools/var_bench.py sym_w8 part19 -- --no-cpu --steps 10 --warmup 2 > $OUT/s20_var.log 2>&1 || exit 5
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 5 --warmup 2 --scale 21 > $OUT/s21_main.log 2>&1 || exit 5
timeout -k 10 300 python3 -u tools/var_bench.py sym_w8 part19 -- --no-cpu --steps 5 --warmup 2 --scale 21 > $OUT/s21_var.log 2>&1 || exit 5
tail -qn1 $OUT/s20_main.log $OUT/s21_main.log | cut -c1-300; cat $OUT/s20_var.log $OUT/s21_var.log | cut -c1-300
for v in "chunks2:CBG_FIBER_CHUNKS=2" "chunks1:CBG_FIBER_CHUNKS=1" "nopipe:CBG_FIBER_PIPE=0"; do
  name=${v%%:*}; envv=${v#*:}
  env $envv TAG=r04e/reh_${name}_s18 PORT=29750 bash tools/gpu_dist_rehearsal.sh 2 18 >> $OUT/rehearsal.txt 2>&1 || exit 6
done
for v in "chunks2:CBG_FIBER_CHUNKS=2" "nopipe:CBG_FIBER_PIPE=0"; do
  name=${v%%:*}; envv=${v#*:}
  env $envv TAG=r04e/reh_${name}_s19 PORT=29760 bash tools/gpu_dist_rehearsal.sh 8 19 >> $OUT/rehearsal.txt 2>&1 || exit 6
done
cat $OUT/rehearsal.txt
