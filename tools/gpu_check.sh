#!/bin/bash
# GPU round-trip used during development (run through gpurun from the repo root):
#   tests -> bench -> rocprofv3 kernel stats.  Every GPU step has its own time limit; the
#   script stops at the first failing step.  Outputs land in gpurun_out/.
# usage: tools/gpu_check.sh [tag] [bench args...]
set -u
TAG=${1:-dev}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/gpu_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 13; }
tail -1 "$OUT/bench.log"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu "$@" > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 4; }
echo "prof ok"
find "$OUT/prof" -name '*kernel_stats.csv' | head -1 | xargs -r head -25 | cut -c1-220
