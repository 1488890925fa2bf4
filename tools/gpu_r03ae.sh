#!/bin/bash
# small-product changes (k_col_stats lanes per column, 8-entry one-lane class): parity, config 5, s20
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ae; mkdir -p $O
true
true
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o run -- python3 tools/bench_configs.py --only 5 > $O/c5p.log 2>&1
python3 tools/kstats.py $O/c5/run_kernel_stats.csv | grep -E "col_stats|num_lane|sym_lane|num_wave|sym_wave" || true
timeout -k 10 240 python3 tools/bench_configs.py --only 5 > $O/c5.log 2>&1
grep -h '^{' $O/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('triple', d['triple_ms'], 'fused', d['fused_rap_ms'], 'restrict', d['restriction_device_ms'])"
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > $O/s20.log 2>&1
tail -1 $O/s20.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('s20', round(d['ms_per_step'],2), d['phases_ms'])"
