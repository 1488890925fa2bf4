#!/bin/bash
# config 4 prune: LDS stage capacity 4096 vs 2048 (kernel stats)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03x; mkdir -p $O
for c in 128 4096; do
CBG_MCL_CAP=$c timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$c -o run -- python3 tools/bench_configs.py --only 4 > $O/c$c.log 2>&1
grep -h '^{' $O/c$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($c, d['expansion_ms'], d['prune_ms'])"
python3 tools/kstats.py $O/c$c/run_kernel_stats.csv | grep -i "mcl"
done
