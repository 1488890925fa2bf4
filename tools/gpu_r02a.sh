#!/bin/bash
# Round-2 GPU pass A (run through gpurun from the repo root): GPU tests, the verified bench, kernel
# stats, PMC counter groups over one s20 product, and a probe of RCCL with two ranks on one GPU.
# Every GPU step has its own time limit; the script stops at the first failing GPU step.
set -u
TAG=${1:-r02a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }

step counters-list
timeout -k 10 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || echo "rocprofv3 -L rc=$?"

step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/gpu_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi

step bench
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 13; }
tail -1 "$OUT/bench.log"

step kernel-stats
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 4; }
find "$OUT/prof" -name '*kernel_stats.csv' | head -1 | xargs -r head -25 | cut -c1-200

i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  step "pmc$i $grp"
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc$i.log"; fi
  case $rc in 124|134|137|139) exit $rc;; esac
done
python3 tools/pmc_summary.py "$OUT/${TAG}_pmc.json" "$OUT"/pmc* > "$OUT/pmc_summary.txt" 2>&1 || true
head -30 "$OUT/pmc_summary.txt"

step rccl-probe
timeout -k 10 120 python3 tools/rccl_probe.py > "$OUT/rccl_probe.log" 2>&1
echo "rccl probe rc=$?"; tail -5 "$OUT/rccl_probe.log"
