#!/bin/bash
# round 5: NT stores + opaque ticket by default; A/B of LDS-staged symbolic row handoff (var rl) at s20 and s21
set -u
OUT=gpurun_out/r05h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 12; }
tail -1 $OUT/bench.log | cut -c1-250
timeout -k 10 500 python3 -u tools/var_bench.py rl -- --no-cpu --steps 10 --scale 20 > $OUT/var.log 2>&1 || { tail -5 $OUT/var.log; exit 11; }
cat $OUT/var.log | cut -c1-300
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 > $OUT/bench_2.log 2>&1 || { tail -5 $OUT/bench_2.log; exit 13; }
tail -1 $OUT/bench_2.log | cut -c1-250
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 5 --scale 21 > $OUT/bench_s21.log 2>&1 || { tail -5 $OUT/bench_s21.log; exit 14; }
tail -1 $OUT/bench_s21.log | cut -c1-250
timeout -k 10 500 python3 -u tools/var_bench.py rl -- --no-cpu --steps 5 --scale 21 > $OUT/var_s21.log 2>&1 || { tail -5 $OUT/var_s21.log; exit 15; }
cat $OUT/var_s21.log | cut -c1-300
timeout -k 10 400 python3 -u -m pytest tests/test_spgemm_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 16; }
tail -1 $OUT/tests.log
