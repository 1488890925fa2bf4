#!/bin/bash
# dev helper: rocprofv3 PMC passes over one bench step (one pass per counter group) + summary
set -u
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
python3 tools/pmc_summary.py "$OUT/${TAG}_pmc.json" "$OUT"/pmc* > "$OUT/pmc_summary.txt" 2>&1 || true
head -3 "$OUT/pmc_summary.txt" | cut -c1-900
