#!/bin/bash
# round 5: heavy-kernel claim scheme A/B (round-4 scheme = var claim0), full-size GPU tests, config 4/5 rank shares
set -u
OUT=gpurun_out/r05e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/var_bench.py claim0 -- --no-cpu --steps 10 --scale 20 > $OUT/var.log 2>&1 || { tail -5 $OUT/var.log; exit 11; }
cat $OUT/var.log | cut -c1-300
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 12; }
tail -1 $OUT/bench.log | cut -c1-250
timeout -k 10 300 python3 -u tools/old_r04/bench.py --no-cpu --steps 10 > $OUT/bench_r04tree.log 2>&1 || { tail -5 $OUT/bench_r04tree.log; exit 13; }
tail -1 $OUT/bench_r04tree.log | cut -c1-250
timeout -k 10 400 python3 -u -m pytest tests/test_fullsize_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests_fullsize.log 2>&1 || { tail -30 $OUT/tests_fullsize.log; exit 14; }
tail -3 $OUT/tests_fullsize.log
timeout -k 10 900 python3 -u tools/rank_share_configs.py > $OUT/rank_share_configs.jsonl 2> $OUT/rank_share_configs.err || { tail -10 $OUT/rank_share_configs.err; exit 15; }
cut -c1-300 $OUT/rank_share_configs.jsonl
