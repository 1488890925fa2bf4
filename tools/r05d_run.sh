#!/bin/bash
# round 5: same-box A/B against the round-4 tree (tools/old_r04), full-size GPU tests, config 4/5 rank shares
set -u
OUT=gpurun_out/r05d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/old_r04/bench.py --no-cpu --steps 10 > $OUT/bench_r04tree.log 2>&1 || { tail -5 $OUT/bench_r04tree.log; exit 11; }
tail -1 $OUT/bench_r04tree.log | cut -c1-250
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 12; }
tail -1 $OUT/bench.log | cut -c1-250
timeout -k 10 300 python3 -u tools/old_r04/bench.py --no-cpu --steps 10 > $OUT/bench_r04tree_2.log 2>&1 || { tail -5 $OUT/bench_r04tree_2.log; exit 13; }
tail -1 $OUT/bench_r04tree_2.log | cut -c1-250
timeout -k 10 400 python3 -u tools/var_bench.py nopf opq opqnt -- --no-cpu --steps 10 --scale 20 > $OUT/var_nopf.log 2>&1 || { tail -5 $OUT/var_nopf.log; exit 16; }
cat $OUT/var_nopf.log | cut -c1-300
timeout -k 10 400 python3 -u -m pytest tests/test_spgemm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_spgemm.log 2>&1 || { tail -20 $OUT/tests_spgemm.log; exit 17; }
tail -1 $OUT/tests_spgemm.log
timeout -k 10 400 python3 -u -m pytest tests/test_fullsize_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests_fullsize.log 2>&1 || { tail -30 $OUT/tests_fullsize.log; exit 14; }
tail -3 $OUT/tests_fullsize.log
timeout -k 10 900 python3 -u tools/rank_share_configs.py > $OUT/rank_share_configs.jsonl 2> $OUT/rank_share_configs.err || { tail -10 $OUT/rank_share_configs.err; exit 15; }
cut -c1-300 $OUT/rank_share_configs.jsonl
