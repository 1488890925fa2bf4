#!/bin/bash
# r04o: heavy threshold variants (nnz(C(:,j)) above which a column becomes units): 4096 (base), 3072, 2048; s20, s21
set -u
OUT=gpurun_out/r04o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/var_bench.py base h3072 h2048 -- --no-cpu --steps 5 --warmup 2 > $OUT/s20.log 2>&1 || { tail -5 $OUT/s20.log; exit 13; }
cat $OUT/s20.log | cut -c1-400
timeout -k 10 500 python -u tools/var_bench.py base h2048 -- --no-cpu --steps 3 --warmup 1 --scale 21 > $OUT/s21.log 2>&1 || { tail -5 $OUT/s21.log; exit 13; }
cat $OUT/s21.log | cut -c1-400
