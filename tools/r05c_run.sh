#!/bin/bash
# round 5: heavy-kernel row words (no wait at the prefetch), merge prefetch in both passes, tuning variants
set -u
OUT=gpurun_out/r05c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_spgemm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_spgemm.log 2>&1 || { tail -20 $OUT/tests_spgemm.log; exit 11; }
tail -1 $OUT/tests_spgemm.log
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 12; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 600 python3 -u tools/var_bench.py rw u4 nt noopt -- --no-cpu --steps 5 --scale 20 > $OUT/var_s20.log 2>&1 || { tail -5 $OUT/var_s20.log; exit 13; }
cat $OUT/var_s20.log | cut -c1-400
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 5 --scale 21 > $OUT/bench_s21.log 2>&1 || { tail -5 $OUT/bench_s21.log; exit 14; }
tail -1 $OUT/bench_s21.log | cut -c1-300
