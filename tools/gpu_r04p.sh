#!/bin/bash
# r04p: rows-known units taken in first-subwindow order (CBG_KNOWN_ORDER) vs column order -- product parity,
# then s20 and s21 bench lines both ways.
set -u
OUT=gpurun_out/r04p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; }
for sc in 20 21; do
  for o in 1 0; do
    CBG_KNOWN_ORDER=$o timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 2 --scale $sc > $OUT/b${sc}_$o.log 2>&1 || { echo "bench $sc $o failed"; tail -3 $OUT/b${sc}_$o.log; exit 13; }
    tail -1 $OUT/b${sc}_$o.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('s$sc order=$o', round(d['ms_per_step'],2), d['phases_ms'], round(d['roofline']['frac'],4), d.get('verified',{}).get('bit_exact'))"
  done
done
