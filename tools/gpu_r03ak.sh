#!/bin/bash
# k_sym_part 16-byte row loads (default) vs dword loads (CBG_SYM_VEC4=0): parity, then s20 A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ak; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in 1 0 1 0; do
CBG_SYM_VEC4=$v timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > $O/s20_$v.log 2>&1
tail -1 $O/s20_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vec', $v, round(d['ms_per_step'],2), d['phases_ms']['symbolic_ms'], d['phases_ms']['heavy_ms'])"
done
