#!/bin/bash
# r04f: the whole GPU test suite on the build with 32-bit symbolic staging (one process, per-test limits).
set -u
OUT=gpurun_out/r04f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1050 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/gpu_tests.log | tail -8; exit $rc
