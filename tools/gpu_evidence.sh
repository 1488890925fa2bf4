#!/bin/bash
# The round's same-build evidence on one MI355X (run from the repo root under gpurun; each step has its own time limit
# inside tools/gpu_steps.sh, and the script stops at the first failure).  TAG names the gpurun_out/ directory and the
# profiles/ files; copy what is to be judged from gpurun_out/TAG into profiles/ afterwards.
#   tools/gpu_evidence.sh TAG local    GPU suite, heavy + whole-product PMC (copied into profiles/ before the bench so
#                                      the bench line's traffic fields come from this build), the N = 1 bench line as
#                                      the driver runs it, rocprofv3 kernel stats, SQ counters
#   tools/gpu_evidence.sh TAG multi    every rank's share of the 8 / 4 / 2-GPU layouts (verified), RCCL rehearsals of
#                                      N = 8 / 4 / 2 at s19 (verified bench lines whose whole-product checksums must
#                                      agree across the layouts) and N = 2 at s18, merge bench, stamps (diag build)
#   tools/gpu_evidence.sh TAG extra    rocprofv3 stats of the s22 2x2x2 rank-0 share, the fiber codec at s21
set -u
T=$1
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
case ${2:-local} in
  local)
    tools/gpu_steps.sh "$T" tests pmc || exit $?
    cp "$OUT/${T}_pmc_heavy.json" "profiles/${T}_pmc_heavy.json" && cp "$OUT/${T}_pmc_product.json" "profiles/${T}_pmc_product.json" || exit 20
    tools/gpu_steps.sh "$T" bench:--steps,20,--warmup,5 prof sq || exit $? ;;
  multi)
    tools/gpu_steps.sh "$T" share:8:22 share:4:21 share:2:21 dist:8:19 dist:4:19 dist:2:19 dist:2:18 || exit $?
    timeout -k 10 300 python3 -u tools/bench_merge.py --scale 20 --reps 3 > "$OUT/merge_s20.log" 2>&1 || exit 30
    if [ -f tools/diag/libcbgpu.so ]; then
      timeout -k 10 300 python3 -u tools/diag_stamps.py 20 > "$OUT/diag_stamps_s20.txt" 2>&1 || exit 31
      timeout -k 10 300 python3 -u tools/diag_known.py > "$OUT/diag_known.txt" 2>&1 || exit 32
    fi ;;
  extra)
    tools/gpu_steps.sh "$T" shareprof:8:22 codec:21 || exit $? ;;
  *) echo "unknown mode $2"; exit 9 ;;
esac
echo "== evidence $T ${2:-local} done"
