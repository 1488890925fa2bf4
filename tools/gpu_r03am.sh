#!/bin/bash
# vector row / (row, value) loads in every hash kernel: parity, s20, config 4
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ao; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py tests/test_mcl_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > $O/s20.log 2>&1
tail -1 $O/s20.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('s20', round(d['ms_per_step'],2), d['phases_ms'])"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 tools/bench_configs.py --only 4 > $O/c4.log 2>&1
grep -h '^{' $O/c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['expansion_ms'], d['product_ms'], d['prune_ms'])"
python3 tools/kstats.py $O/c4/run_kernel_stats.csv | head -8 || true
