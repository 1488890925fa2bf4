#!/bin/bash
# r04k: one-pass flat merge with relaxed look-back states -- parity, then the s20 1x1x2 merge bench:
# one pass (values staged in LDS), two passes, one pass without the value stage (tools/var/vs0), kernel trace.
set -u
OUT=gpurun_out/r04k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -k "merge" -x -q --timeout 60 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; }
run() { timeout -k 10 240 python -u tools/bench_merge.py --scale 20 --reps 3 "$@" 2> $OUT/$tag.err > $OUT/$tag.json || { echo "merge bench $tag failed"; tail -5 $OUT/$tag.err; exit 4; }; cut -c1-300 $OUT/$tag.json; }
tag=one_vs; run
tag=two_vs; CBG_MERGE_ONEPASS=0 run
tag=one_novs; CBG_MERGE_VSTAGE=0 run --lib tools/var/vs0/libcbgpu.so
tag=two_novs; CBG_MERGE_ONEPASS=0 CBG_MERGE_VSTAGE=0 run --lib tools/var/vs0/libcbgpu.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_merge.py --scale 20 --reps 2 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $OUT/prof.log; exit 5; }
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv | grep -iE "merge|split" | head -6
