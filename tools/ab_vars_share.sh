#!/bin/bash
# A/B of compile-time variants (tools/var/<name>/libcbgpu.so, `main` = this build) at s20 (twice) and on the s22 2x2x2
# rank shares 0 and 4, one process per variant, same box:   tools/ab_vars_share.sh TAG name [name ...]
set -u
T=$1; shift
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 600 python3 -u tools/var_bench.py main "$@" -- --no-cpu --steps 10 --scale 20 > "$OUT/var_s20_$r.log" 2>&1 || { tail -5 "$OUT/var_s20_$r.log"; exit 11; }
  cut -c1-300 "$OUT/var_s20_$r.log"
done
timeout -k 10 900 python3 -u tools/var_bench.py main "$@" -- --rank-share 0,4 --gpus-virtual 8 --scale 22 --no-cpu > "$OUT/var_share22.log" 2>&1 || { tail -5 "$OUT/var_share22.log"; exit 12; }
cut -c1-300 "$OUT/var_share22.log"
