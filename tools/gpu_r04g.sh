#!/bin/bash
# r04g: flat tiled two-way merge -- parity (merge tests, fiber / layout tests that merge), then the s20 1x1x2
# merge bench flat vs per-column, and a kernel trace of the flat one.
set -u
OUT=gpurun_out/r04g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py -k "merge" -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -k "fiber or summa_layouts or reference_fixtures_through" -x -q --timeout 150 --timeout-method thread > $OUT/dist.log 2>&1
rc=$?; tail -2 $OUT/dist.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  CBG_MERGE_FLAT=$f timeout -k 10 240 python -u tools/bench_merge.py --scale 20 --reps 3 > $OUT/merge_flat$f.json 2> $OUT/merge_flat$f.err || { echo "merge bench $f failed"; tail -5 $OUT/merge_flat$f.err; exit 4; }
  cut -c1-400 $OUT/merge_flat$f.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_merge.py --scale 20 --reps 2 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $OUT/prof.log; exit 5; }
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv | grep -iE "merge|split|scan" | head -12
