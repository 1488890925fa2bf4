#!/bin/bash
# r04j: one-pass flat merge (decoupled look-back) -- parity both ways, s20 1x1x2 merge bench one-pass vs two-pass,
# kernel trace, then the fiber / layout tests that merge.
set -u
OUT=gpurun_out/r04j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -k "merge" -x -q --timeout 60 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; }
CBG_MERGE_ONEPASS=0 timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -k "merge" -x -q --timeout 60 --timeout-method thread > $OUT/tests0.log 2>&1
rc=$?; tail -1 $OUT/tests0.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  CBG_MERGE_ONEPASS=$f timeout -k 10 240 python -u tools/bench_merge.py --scale 20 --reps 3 > $OUT/merge_one$f.json 2> $OUT/merge_one$f.err || { echo "merge bench $f failed"; tail -5 $OUT/merge_one$f.err; exit 4; }
  cut -c1-330 $OUT/merge_one$f.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_merge.py --scale 20 --reps 2 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $OUT/prof.log; exit 5; }
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv | grep -iE "merge|split" | head -6
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -k "fiber or summa_layouts or reference_fixtures_through" -x -q --timeout 150 --timeout-method thread > $OUT/dist.log 2>&1
rc=$?; tail -2 $OUT/dist.log; exit $rc
