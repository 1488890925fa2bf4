#!/bin/bash
# Which unit bounds k_num_heavy_known: texture address / data / L1 counters (one pass per group)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ad; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1
grep -oE "\b(TA|TD|TCP)_[A-Z0-9_]+" $O/avail.txt | sort -u > $O/names.txt
wc -l $O/names.txt
i=0
for grp in "TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS" "TD_TD_BUSY TD_TC_STALL" "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_GATE_EN1" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/p$i.log 2>&1
  echo "pass $i rc=$?"
done
