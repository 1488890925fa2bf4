#!/bin/bash
# r04c: drop-in tests (RestrictionOp at q=2 after the collective-free device binding), the chunked fiber pipeline
# (fiber formats, RCCL fixtures at world 2/8, MCL over RCCL), rank shares with the new wire accounting, the merge A/B,
# the 8-wave symbolic A/B, one-GPU RCCL rehearsals (1x1x2 s18, 2x2x2 s19: chunked / one chunk / unpipelined).
set -u
OUT=gpurun_out/r04c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dropin.py tests/test_dist_gpu.py -x -v --timeout 170 --timeout-method thread \
  -k "dropin or fiber or rccl_multirank or mcl_expansion" > $OUT/tests.log 2>&1
rc=$?; grep -cE "PASSED" $OUT/tests.log; grep -E "FAILED|Error" $OUT/tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --rank-share 0,4 --gpus-virtual 8 --scale 22 > $OUT/rank_share_s22.jsonl 2> $OUT/rank_share.err || { tail -5 $OUT/rank_share.err; exit 13; }
timeout -k 10 600 python -u bench.py --rank-share all --gpus-virtual 2 --scale 21 > $OUT/rank_share_s21_n2.jsonl 2> $OUT/rank_share2.err || { tail -5 $OUT/rank_share2.err; exit 13; }
timeout -k 10 300 python3 tools/bench_merge.py --scale 20 --reps 3 --lib tools/var/merge_old/libcbgpu.so > $OUT/merge_old.log 2>&1 || { tail -5 $OUT/merge_old.log; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mprof -o run -- python3 tools/bench_merge.py --scale 20 --reps 3 > $OUT/merge.log 2>&1 || { tail -5 $OUT/merge.log; exit 4; }
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 --warmup 2 > $OUT/s20_main.log 2>&1 || exit 5
timeout -k 10 300 python3 -u tools/var_bench.py sym_w8 -- --no-cpu --steps 10 --warmup 2 > $OUT/s20_symw8.log 2>&1 || exit 5
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 5 --warmup 2 --scale 21 > $OUT/s21_main.log 2>&1 || exit 5
timeout -k 10 300 python3 -u tools/var_bench.py sym_w8 -- --no-cpu --steps 5 --warmup 2 --scale 21 > $OUT/s21_symw8.log 2>&1 || exit 5
timeout -k 10 300 python3 -u tools/var_bench.py part19 -- --no-cpu --steps 5 --warmup 2 --scale 21 > $OUT/s21_part19.log 2>&1 || exit 5
timeout -k 10 300 python3 -u tools/var_bench.py part19 -- --no-cpu --steps 10 --warmup 2 > $OUT/s20_part19.log 2>&1 || exit 5
for v in "chunks2:CBG_FIBER_CHUNKS=2" "chunks1:CBG_FIBER_CHUNKS=1" "nopipe:CBG_FIBER_PIPE=0"; do
  name=${v%%:*}; envv=${v#*:}
  env $envv TAG=r04c/reh_${name}_s18 PORT=29750 bash tools/gpu_dist_rehearsal.sh 2 18 >> $OUT/rehearsal.txt 2>&1 || exit 6
done
for v in "chunks2:CBG_FIBER_CHUNKS=2" "nopipe:CBG_FIBER_PIPE=0"; do
  name=${v%%:*}; envv=${v#*:}
  env $envv TAG=r04c/reh_${name}_s19 PORT=29760 bash tools/gpu_dist_rehearsal.sh 8 19 >> $OUT/rehearsal.txt 2>&1 || exit 6
done
cat $OUT/rehearsal.txt
