#!/bin/bash
set -u
TAG=${1:-r02g}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/t.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log" | cut -c1-600; exit 13; }
python3 -c "import json;d=json.loads(open('$OUT/bench.log').read().splitlines()[-1]);print('bench', d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d['heavy_items'], d.get('verified',{}).get('bit_exact'))"
timeout -k 10 300 python3 -u tools/diag_stamps.py 20 > "$OUT/stamps.log" 2>&1; echo "stamps rc=$?"; head -8 "$OUT/stamps.log"
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((${i:-0}+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
python3 tools/pmc_summary.py "$OUT/${TAG}_pmc.json" "$OUT"/pmc* > "$OUT/pmc_summary.txt" 2>&1 || true
head -4 "$OUT/pmc_summary.txt" | cut -c1-700
