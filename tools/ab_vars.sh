#!/bin/bash
# A/B of compile-time variants (tools/var/<name>/libcbgpu.so) against this build at s20 and s21, same box:
#   tools/ab_vars.sh TAG name [name ...]
set -u
T=$1; shift
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
for sc in 20 21; do
  timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 --scale $sc > "$OUT/bench_s$sc.log" 2>&1 || { tail -5 "$OUT/bench_s$sc.log"; exit 11; }
  python3 -c "
import json
L=[l for l in open('$OUT/bench_s$sc.log') if l.startswith('{')]
d=json.loads(L[-1]); print('main s$sc', round(d['ms_per_step'],2), d['phases_ms'], round(d['roofline']['frac'],3))"
  timeout -k 10 900 python3 -u tools/var_bench.py "$@" -- --no-cpu --steps 10 --scale $sc > "$OUT/var_s$sc.log" 2>&1 || { tail -5 "$OUT/var_s$sc.log"; exit 12; }
  cut -c1-300 "$OUT/var_s$sc.log"
done
