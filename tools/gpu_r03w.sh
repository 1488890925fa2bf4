#!/bin/bash
# MCL one-histogram selection: parity tests, then config 4 kernel stats for the new and the radix selection.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mcl_gpu.py tests/test_dist_gpu.py -k "mcl or prune or memeff" -x -q --timeout 120 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }; tail -2 $O/t.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fast -o run -- python3 tools/bench_configs.py --only 4 > $O/fast.log 2>&1
CBG_MCL_RADIX=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/radix -o run -- python3 tools/bench_configs.py --only 4 > $O/radix.log 2>&1
grep -h '^{' $O/fast.log $O/radix.log || true
for v in fast radix; do f=$(find $O/$v -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py "$f" 2>/dev/null | grep -i "mcl\|num_block<.*13" || true; done
