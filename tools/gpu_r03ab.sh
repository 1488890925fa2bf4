#!/bin/bash
# rows-known units in subwindow-major order (CBG_KNOWN_ORDER=1) vs column order: parity, s20 and s21
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ab; mkdir -p $O
CBG_KNOWN_ORDER=1 timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for sc in 20 21; do
for o in 0 1; do
CBG_KNOWN_ORDER=$o timeout -k 10 400 python3 -u bench.py --scale $sc --steps 3 --warmup 1 --no-cpu > $O/s${sc}_o$o.log 2>&1
tail -1 $O/s${sc}_o$o.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($sc, $o, round(d['ms_per_step'],2), d['phases_ms']['heavy_ms'], round(d['roofline']['frac'],4))"
done
done
