#!/bin/bash
# small products (config 5 RᵀAR) after a host-path change: GPU suite, config 5 timing + kernel stats, the s20 line
set -u
OUT=gpurun_out/${1:-small}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -20 "$OUT/gpu_tests.log"; exit 11; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python3 -u tools/bench_configs.py --only 5 --reps 10 > "$OUT/config5.jsonl" 2>&1 || { tail -5 "$OUT/config5.jsonl"; exit 12; }
cut -c1-900 "$OUT/config5.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof5" -o c5 -- python3 -u tools/bench_configs.py --only 5 --reps 10 > "$OUT/config5_prof.log" 2>&1 || { tail -5 "$OUT/config5_prof.log"; exit 13; }
timeout -k 10 300 python3 -u bench.py > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 14; }
tail -1 "$OUT/bench.log" | cut -c1-300
