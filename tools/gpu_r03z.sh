#!/bin/bash
# Galerkin: parity tests, then config 5 with kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mcl_gpu.py -k "galerkin or restriction or transpose" -x -q --timeout 120 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o run -- python3 tools/bench_configs.py --only 5 > $O/c5.log 2>&1
grep -h '^{' $O/c5.log | cut -c1-1500
python3 tools/kstats.py $O/c5/run_kernel_stats.csv | grep -i "rap\|mt_draw"
