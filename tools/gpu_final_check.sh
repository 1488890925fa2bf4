#!/bin/bash
# final-tree check as the driver runs it: smoke(), the default bench line (no flags), and the 2x2 (N = 4) RCCL rehearsal
set -u
OUT=gpurun_out/${1:-final}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 11; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench_default.log" 2>&1 || { tail -5 "$OUT/bench_default.log"; exit 12; }
tail -1 "$OUT/bench_default.log" | cut -c1-300
tools/gpu_steps.sh "${1:-final}" dist:4:20 || exit $?
