#!/bin/bash
# dev helper: a chosen subset of GPU tests, then one bench line.
# usage: tools/gpu_quick2.sh <tag> "<pytest selection args>" [bench args...]
set -u
TAG=${1:-q}; SEL=${2:-tests}; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v -s --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" "$OUT/t.log" | tail -40 | cut -c1-200; tail -2 "$OUT/t.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log" | cut -c1-600; exit 13; }
tail -1 "$OUT/bench.log" | cut -c1-3000
