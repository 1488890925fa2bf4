#!/bin/bash
# s21 on one GPU (per-rank size of the N = 2, 4 lines) and config 5 without the profiler
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03aa; mkdir -p $O
timeout -k 10 400 python3 -u bench.py --scale 21 --steps 3 --warmup 1 --no-cpu > $O/s21.log 2>&1
tail -1 $O/s21.log | cut -c1-1200
timeout -k 10 240 python3 tools/bench_configs.py --only 5 > $O/c5.log 2>&1
grep -h '^{' $O/c5.log | cut -c1-1500
