#!/bin/bash
# Round evidence in one gpurun call (run from the repo root):
#   GPU tests -> bench line -> rocprofv3 kernel stats -> heavy-kernel HBM traffic (FETCH/WRITE passes)
#   -> limiter counters (SQ groups) over one bench product.
# Every GPU step has its own limit; the script stops at the first step that fails.
# usage: tools/gpu_round.sh <tag> [--no-tests | --tests-only]   (one gpurun call is capped at 20 minutes: the whole
# GPU suite and the profiling passes go in separate calls)
set -u
TAG=${1:-r02}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${1:-}" != "--no-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/gpu_tests.log"
  [ $rc -eq 0 ] || exit $rc
fi
[ "${1:-}" = "--tests-only" ] && exit 0
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log" | cut -c1-600; exit 13; }
tail -1 "$OUT/bench.log" | cut -c1-1500
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 4; }
echo "prof ok"
timeout -k 10 600 python3 -u tools/pmc_heavy.py run "$TAG" 20 > "$OUT/pmc_heavy.log" 2>&1 || { echo "pmc_heavy failed"; tail -5 "$OUT/pmc_heavy.log"; exit 5; }
tail -1 "$OUT/pmc_heavy.log" | cut -c1-600
timeout -k 10 600 python3 -u tools/pmc_heavy.py product "$TAG" 20 > "$OUT/pmc_product.log" 2>&1 || { echo "pmc product failed"; tail -5 "$OUT/pmc_product.log"; exit 6; }
tail -1 "$OUT/pmc_product.log" | cut -c1-600
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT/sq$i" -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu > "$OUT/sq$i.log" 2>&1
  rc=$?; echo "sq $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py "$OUT/${TAG}_sq.json" "$OUT"/sq1 "$OUT"/sq2 > "$OUT/sq_summary.txt" 2>&1 || true
head -4 "$OUT/sq_summary.txt" | cut -c1-900
