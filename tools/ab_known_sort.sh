#!/bin/bash
# A/B of the rows-known units in first-subwindow order (CBG_KNOWN_SORT=1) on one build: parity first, then s20, s21 and
# the s22 2x2x2 rank-0 share with and without
set -u
OUT=gpurun_out/${1:-ksort}
mkdir -p "$OUT"
export TMPDIR=/tmp
CBG_KNOWN_SORT=1 timeout -k 10 400 python3 -u -m pytest tests/test_spgemm_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests_sorted.log" 2>&1 || { tail -20 "$OUT/tests_sorted.log"; exit 11; }
tail -1 "$OUT/tests_sorted.log"
for sc in 20 21; do
  for ks in 0 1; do
    CBG_KNOWN_SORT=$ks timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 --scale $sc > "$OUT/bench_s${sc}_sort$ks.log" 2>&1 || { tail -5 "$OUT/bench_s${sc}_sort$ks.log"; exit 12; }
    python3 -c "
import json
L=[l for l in open('$OUT/bench_s${sc}_sort$ks.log') if l.startswith('{')]
d=json.loads(L[-1]); print('s$sc sort$ks', round(d['ms_per_step'],2), d['phases_ms'], round(d['roofline']['frac'],3))"
  done
done
for ks in 0 1; do
  CBG_KNOWN_SORT=$ks timeout -k 10 300 python3 -u bench.py --rank-share 0 --gpus-virtual 8 --scale 22 > "$OUT/share_s22_r0_sort$ks.jsonl" 2> "$OUT/share_s22_r0_sort$ks.err" || { tail -5 "$OUT/share_s22_r0_sort$ks.err"; exit 13; }
  python3 -c "
import json
L=[json.loads(l) for l in open('$OUT/share_s22_r0_sort$ks.jsonl') if l.startswith('{')]
d=L[-1]; print('s22 rank0 sort$ks local', d['local_ms'], 'heavy', d['heavy_ms'], 'sym', d['symbolic_ms'], 'bit_exact', d['verified']['bit_exact'])"
done
