#!/bin/bash
# k_num_heavy_known paired (row, value) loads (CBG_NUM_VEC2) A/B + parity with the default build
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03al; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 800 python3 -u tools/var_bench.py novec2 vec2 novec2 vec2 -- --no-cpu --steps 5 > $O/var.log 2>&1
cut -c1-260 $O/var.log
