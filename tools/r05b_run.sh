#!/bin/bash
# round 5: deferred 16-bit row reconstruction in the heavy kernel + merge count-pass row prefetch (A/B)
set -u
OUT=gpurun_out/r05b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_spgemm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_spgemm.log 2>&1 || { tail -20 $OUT/tests_spgemm.log; exit 11; }
tail -1 $OUT/tests_spgemm.log
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 12; }
tail -1 $OUT/bench.log | cut -c1-200
for pf in 0 1 2; do
  CBG_MERGE_PF=$pf timeout -k 10 300 python3 -u tools/bench_merge.py --scale 20 --reps 3 > $OUT/merge_pf$pf.log 2>&1 || { tail -5 $OUT/merge_pf$pf.log; exit 13; }
  tail -1 $OUT/merge_pf$pf.log | cut -c1-400
done
timeout -k 10 300 python3 -u tools/diag_known.py > $OUT/diag_known.txt 2>&1 || { tail -5 $OUT/diag_known.txt; exit 14; }
cat $OUT/diag_known.txt
