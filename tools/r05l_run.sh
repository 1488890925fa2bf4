#!/bin/bash
# round 5: A/B of paired 16-byte value stores in the rows-known kernel (var vp) and 2^19-row symbolic parts with 1024-thread workgroups (var p19), at s20 and s21
set -u
OUT=gpurun_out/r05l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/var_bench.py vp p19 -- --no-cpu --steps 10 --scale 20 > $OUT/var.log 2>&1 || { tail -5 $OUT/var.log; exit 11; }
cat $OUT/var.log | cut -c1-300
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 12; }
tail -1 $OUT/bench.log | cut -c1-250
timeout -k 10 500 python3 -u tools/var_bench.py vp p19 -- --no-cpu --steps 5 --scale 21 > $OUT/var_s21.log 2>&1 || { tail -5 $OUT/var_s21.log; exit 13; }
cat $OUT/var_s21.log | cut -c1-300
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 5 --scale 21 > $OUT/bench_s21.log 2>&1 || { tail -5 $OUT/bench_s21.log; exit 14; }
tail -1 $OUT/bench_s21.log | cut -c1-250
