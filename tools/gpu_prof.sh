#!/bin/bash
# dev helper: one bench line + rocprofv3 kernel stats (top kernels printed).  usage: tools/gpu_prof.sh <tag> [bench args]
set -u
TAG=${1:-prof}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --no-cpu "$@" > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log" | cut -c1-600; exit 13; }
python3 -c "import json;d=json.loads(open('$OUT/bench.log').read().splitlines()[-1]);print('bench', d['ms_per_step'], d['phases_ms'], round(d['roofline']['frac'],4))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu "$@" > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 4; }
python3 tools/kstats.py "$OUT/prof/run_kernel_stats.csv" 2>/dev/null | head -16 || true
