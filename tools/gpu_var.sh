#!/bin/bash
# dev helper: bench tuning variants (tools/var/<name>/libcbgpu.so) on the same input.  usage: tools/gpu_var.sh tag name...
set -u
TAG=$1; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/var_bench.py "$@" -- --no-cpu --steps 5 > gpurun_out/$TAG/var.log 2>&1
rc=$?; cut -c1-300 gpurun_out/$TAG/var.log; exit $rc
