#!/bin/bash
# GPU tests, then the bench with and without the symbolic->numeric row handoff, then kernel stats.
set -u
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/gpu_tests.log" | cut -c1-400
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log" | cut -c1-600; exit 13; }
python3 -c "import json;d=json.loads(open('$OUT/bench.log').read().splitlines()[-1]);print('handoff', d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d.get('verified'))"
CBG_ROW_HANDOFF=0 timeout -k 10 600 python -u bench.py --no-cpu > "$OUT/bench_off.log" 2>&1 || { echo "bench off failed"; exit 13; }
python3 -c "import json;d=json.loads(open('$OUT/bench_off.log').read().splitlines()[-1]);print('no handoff', d['ms_per_step'], d['phases_ms'], d['roofline']['frac'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; exit 4; }
find "$OUT/prof" -name '*kernel_stats.csv' | head -1 | xargs -r head -12 | cut -c1-160
