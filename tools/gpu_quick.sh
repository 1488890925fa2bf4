#!/bin/bash
# dev helper: spgemm GPU tests + one bench line (+ stamps with STAMPS=1)
set -u
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/t.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log" | cut -c1-600; exit 13; }
python3 -c "import json;d=json.loads(open('$OUT/bench.log').read().splitlines()[-1]);print('bench', d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d['heavy_items'], d.get('verified',{}).get('bit_exact'))"
if [ -n "${STAMPS:-}" ]; then
  timeout -k 10 300 python3 -u tools/diag_stamps.py 20 > "$OUT/stamps.log" 2>&1; echo "stamps rc=$?"; head -8 "$OUT/stamps.log"
fi
