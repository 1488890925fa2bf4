#!/bin/bash
# r04l: every rank's share of the mandated layouts on this one GPU with the flat merge:
# 2x2x2 at s22 (N = 8), 1x1x2 at s21 (N = 2), 2x2 at s21 (N = 4); then the N = 1 bench line.
set -u
OUT=gpurun_out/r04l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -k "merge" -x -q --timeout 60 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 240 python -u tools/bench_merge.py --scale 20 --reps 3 > $OUT/merge_s20.json 2> $OUT/merge.err || { tail -5 $OUT/merge.err; exit 4; }
cut -c1-300 $OUT/merge_s20.json
timeout -k 10 420 python -u bench.py --rank-share all --gpus-virtual 8 --scale 22 > $OUT/rank_share_s22_n8.jsonl 2> $OUT/rs8.err
rc=$?; cut -c1-260 $OUT/rank_share_s22_n8.jsonl; [ $rc -eq 0 ] || { tail -5 $OUT/rs8.err; exit $rc; }
timeout -k 10 240 python -u bench.py --rank-share all --gpus-virtual 2 --scale 21 > $OUT/rank_share_s21_n2.jsonl 2> $OUT/rs2.err
rc=$?; cut -c1-260 $OUT/rank_share_s21_n2.jsonl; [ $rc -eq 0 ] || { tail -5 $OUT/rs2.err; exit $rc; }
timeout -k 10 240 python -u bench.py --rank-share all --gpus-virtual 4 --scale 21 > $OUT/rank_share_s21_n4.jsonl 2> $OUT/rs4.err
rc=$?; cut -c1-260 $OUT/rank_share_s21_n4.jsonl; [ $rc -eq 0 ] || { tail -5 $OUT/rs4.err; exit $rc; }
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log | cut -c1-600; exit 13; }
tail -1 $OUT/bench.log | cut -c1-600
