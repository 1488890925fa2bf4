#!/bin/bash
# r04b: varint fiber formats (distributed GPU tests over gloo and RCCL), rank shares with the new wire accounting
# (2x2x2 s22 ranks 0 and 4, 1x1x2 s21 both ranks), the two-way merge's kernel stats + SQ counters at s20.
set -u
OUT=gpurun_out/r04b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_dist_gpu.py tests/test_dropin.py -x -v --timeout 300 --timeout-method thread > $OUT/dist_tests.log 2>&1
rc=$?; grep -E "passed|failed|PASS|FAIL" $OUT/dist_tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --rank-share 0,4 --gpus-virtual 8 --scale 22 > $OUT/rank_share_s22.jsonl 2> $OUT/rank_share.err || { tail -5 $OUT/rank_share.err; exit 13; }
cut -c1-900 $OUT/rank_share_s22.jsonl
timeout -k 10 600 python -u bench.py --rank-share all --gpus-virtual 2 --scale 21 > $OUT/rank_share_s21_n2.jsonl 2> $OUT/rank_share2.err || { tail -5 $OUT/rank_share2.err; exit 13; }
cut -c1-900 $OUT/rank_share_s21_n2.jsonl
timeout -k 10 300 python3 tools/bench_merge.py --scale 20 --reps 3 --lib tools/var/merge_old/libcbgpu.so > $OUT/merge_old.log 2>&1 || { tail -5 $OUT/merge_old.log; exit 4; }
tail -1 $OUT/merge_old.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mprof -o run -- python3 tools/bench_merge.py --scale 20 --reps 3 > $OUT/merge.log 2>&1 || { tail -5 $OUT/merge.log; exit 4; }
tail -1 $OUT/merge.log | cut -c1-600
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $OUT/msq1 -o run -- python3 tools/bench_merge.py --scale 20 --reps 1 > $OUT/msq1.log 2>&1
echo "msq1 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $OUT/msq2 -o run -- python3 tools/bench_merge.py --scale 20 --reps 1 > $OUT/msq2.log 2>&1
echo "msq2 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/mfetch -o run -- python3 tools/bench_merge.py --scale 20 --reps 1 > $OUT/mfetch.log 2>&1
echo "mfetch rc=$?"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/mwrite -o run -- python3 tools/bench_merge.py --scale 20 --reps 1 > $OUT/mwrite.log 2>&1
echo "mwrite rc=$?"
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 --warmup 2 > $OUT/s20_main.log 2>&1 && tail -1 $OUT/s20_main.log | cut -c1-900
timeout -k 10 300 python3 -u tools/var_bench.py sym_w8 -- --no-cpu --steps 10 --warmup 2 > $OUT/s20_symw8.log 2>&1; tail -2 $OUT/s20_symw8.log | cut -c1-900
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 5 --warmup 2 --scale 21 > $OUT/s21_main.log 2>&1 && tail -1 $OUT/s21_main.log | cut -c1-900
timeout -k 10 300 python3 -u tools/var_bench.py sym_w8 -- --no-cpu --steps 5 --warmup 2 --scale 21 > $OUT/s21_symw8.log 2>&1; tail -2 $OUT/s21_symw8.log | cut -c1-900
