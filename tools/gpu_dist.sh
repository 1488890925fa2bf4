#!/bin/bash
# distributed GPU tests only (gloo ranks sharing cuda:0, libcbgpu native grid)
set -u
TAG=${1:-dist}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -v --timeout 300 --timeout-method thread -x > "$OUT/dist_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 "$OUT/dist_tests.log" | cut -c1-300
