#!/bin/bash
# One gpurun call as a list of steps (run from the repo root); every GPU step has its own time limit and the
# script stops at the first step that fails (exit 10 + step index: never 2 or 3, which gpurun reserves).
#   tools/gpu_steps.sh <tag> <step> [<step> ...]
# steps:
#   tests              the whole -m gpu suite            tests:<expr>   pytest -m gpu -k <expr>
#   bench              N = 1 bench line (configs[1])     bench:<args>   bench.py with extra args (',' = ' ')
#   dist:<N>:<scale>   N ranks on this one GPU over libcbgpu's RCCL grid (RCCL sockets), verified bench line
#   launch:<N>:<scale> the same, started as `bench.py --gpus N` (the script launches its N ranks itself)
#   share:<N>:<scale>  every rank's share of the N-GPU layout at full size, verified (bench.py --rank-share)
#   codec:<scale>      the fiber wire codec on the 1x1x2 message (tools/bench_codec.py) + its rocprofv3 kernel stats
#   shareprof:<N>:<s>  rocprofv3 kernel stats of rank 0's share of the N-GPU layout at scale s
#   var:<a,b,..>:<s>   tuning variants tools/var/<name>/libcbgpu.so on the N = 1 bench at scale s (var_bench.py)
#   prof               rocprofv3 kernel stats of the bench (5 timed products)
#   pmc                heavy-kernel and whole-product HBM bytes (tools/pmc_heavy.py, one counter per pass)
#   sq                 SQ limiter counters (two groups) over one product
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
fail() { echo "step $i ($1) failed rc=$2"; exit $((10 + i)); }
for step in "$@"; do
  i=$((i + 1))
  IFS=: read -r kind a b <<< "$step"
  echo "== step $i: $step ($(date +%T))"
  case $kind in
    tests)
      if [ -n "${a:-}" ]; then K=(-k "$a"); else K=(); fi
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA "${K[@]}" --timeout 300 --timeout-method thread \
        > "$OUT/gpu_tests${a:+_$a}.log" 2>&1
      rc=$?; tail -2 "$OUT/gpu_tests${a:+_$a}.log"
      [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" "$OUT/gpu_tests${a:+_$a}.log" | head -20; fail "$step" $rc; } ;;
    bench)
      extra=${a//,/ }
      timeout -k 10 600 python -u bench.py $extra > "$OUT/bench${a:+_${a//[ ,=-]/}}.log" 2>&1 || \
        { tail -5 "$OUT/bench${a:+_${a//[ ,=-]/}}.log" | cut -c1-800; fail "$step" 1; }
      tail -1 "$OUT/bench${a:+_${a//[ ,=-]/}}.log" | cut -c1-1200 ;;
    dist)
      CBG_DIST_BACKEND=${BACKEND:-rccl-net} timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node "$a" --master-addr 127.0.0.1 --master-port $((29600 + i)) bench.py --gpus "$a" \
        --steps ${STEPS:-3} --warmup 1 --scale "$b" > "$OUT/dist_n${a}_s${b}.log" 2>&1
      rc=$?; grep '^{' "$OUT/dist_n${a}_s${b}.log" | tail -1 | cut -c1-1500
      [ $rc -eq 0 ] || { grep -v '^{' "$OUT/dist_n${a}_s${b}.log" | tail -8 | cut -c1-400; fail "$step" $rc; } ;;
    launch)   # the same rehearsal started the way the driver may start it: `bench.py --gpus N`, no WORLD_SIZE
      CBG_DIST_BACKEND=${BACKEND:-rccl-net} timeout -k 10 600 python3 bench.py --gpus "$a" \
        --steps ${STEPS:-3} --warmup 1 --scale "$b" > "$OUT/launch_n${a}_s${b}.log" 2> "$OUT/launch_n${a}_s${b}.err"
      rc=$?; cut -c1-1500 "$OUT/launch_n${a}_s${b}.log"
      [ $rc -eq 0 ] && [ "$(grep -c . "$OUT/launch_n${a}_s${b}.log")" = 1 ] || \
        { tail -8 "$OUT/launch_n${a}_s${b}.err" | cut -c1-400; fail "$step" $rc; } ;;
    share)
      timeout -k 10 900 python -u bench.py --rank-share all --gpus-virtual "$a" --scale "$b" \
        > "$OUT/rank_share_s${b}_n${a}.jsonl" 2> "$OUT/rank_share_s${b}_n${a}.err"
      rc=$?; cut -c1-400 "$OUT/rank_share_s${b}_n${a}.jsonl"
      [ $rc -eq 0 ] || { tail -8 "$OUT/rank_share_s${b}_n${a}.err"; fail "$step" $rc; } ;;
    cfgshare)   # cfgshare:<configs>:<gpus list with '.' for ','>  (MCL_N env: graph size) configs 4/5 rank shares
      timeout -k 10 1000 python3 -u tools/rank_share_configs.py --configs "$a" --gpus "${b//./,}" \
        --mcl-n "${MCL_N:-1048576}" > "$OUT/cfgshare_${a//,/}_${b//./}.jsonl" 2> "$OUT/cfgshare_${a//,/}_${b//./}.err"
      rc=$?; grep '^{' "$OUT/cfgshare_${a//,/}_${b//./}.jsonl" | cut -c1-300
      [ $rc -eq 0 ] || { tail -8 "$OUT/cfgshare_${a//,/}_${b//./}.err"; fail "$step" $rc; } ;;
    overlap)   # overlap:<N>:<scale>  own-half product || fiber codec on one GPU (tools/overlap_probe.py), ranks 0
      timeout -k 10 600 python3 -u tools/overlap_probe.py --gpus-virtual "$a" --scale "$b" > "$OUT/overlap_n${a}_s${b}.json" \
        2> "$OUT/overlap_n${a}_s${b}.err" || { tail -8 "$OUT/overlap_n${a}_s${b}.err"; fail "$step" 1; }
      cut -c1-900 "$OUT/overlap_n${a}_s${b}.json" ;;
    codec)
      timeout -k 10 300 python -u tools/bench_codec.py --scale "${a:-21}" > "$OUT/codec_s${a:-21}.json" 2>&1 || \
        { tail -5 "$OUT/codec_s${a:-21}.json"; fail "$step" 1; }
      cut -c1-600 "$OUT/codec_s${a:-21}.json"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/codec_prof" -o run -- \
        python3 tools/bench_codec.py --scale "${a:-21}" --reps 1 > "$OUT/codec_prof.log" 2>&1 || { tail -5 "$OUT/codec_prof.log"; fail "$step" 2; } ;;
    shareprof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/shareprof_s${b}_n${a}" -o run -- \
        python3 bench.py --rank-share 0 --gpus-virtual "$a" --scale "$b" > "$OUT/shareprof_s${b}_n${a}.log" 2>&1 || \
        { tail -8 "$OUT/shareprof_s${b}_n${a}.log"; fail "$step" 1; }
      grep '^{' "$OUT/shareprof_s${b}_n${a}.log" | cut -c1-300 ;;
    var)
      timeout -k 10 600 python3 -u tools/var_bench.py ${a//,/ } -- --no-cpu --steps 3 --scale "${b:-20}" \
        > "$OUT/var_s${b:-20}.log" 2>&1 || { tail -5 "$OUT/var_s${b:-20}.log"; fail "$step" 1; }
      cut -c1-400 "$OUT/var_s${b:-20}.log" ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; fail prof 1; }
      tail -1 "$OUT/prof.log" | cut -c1-400 ;;
    pmc)
      timeout -k 10 600 python3 -u tools/pmc_heavy.py run "$TAG" 20 > "$OUT/pmc_heavy.log" 2>&1 || \
        { tail -5 "$OUT/pmc_heavy.log"; fail pmc 1; }
      tail -1 "$OUT/pmc_heavy.log" | cut -c1-600
      timeout -k 10 600 python3 -u tools/pmc_heavy.py product "$TAG" 20 > "$OUT/pmc_product.log" 2>&1 || \
        { tail -5 "$OUT/pmc_product.log"; fail pmc 2; }
      tail -1 "$OUT/pmc_product.log" | cut -c1-600 ;;
    sq)
      j=0
      for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
                 "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
        j=$((j + 1))
        timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT/sq$j" -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu > "$OUT/sq$j.log" 2>&1 || fail "sq $j" 1
      done
      python3 tools/pmc_summary.py "$OUT/${TAG}_sq.json" "$OUT"/sq1 "$OUT"/sq2 > "$OUT/sq_summary.txt" 2>&1 || true
      head -4 "$OUT/sq_summary.txt" | cut -c1-900 ;;
    *) echo "unknown step $step"; exit 9 ;;
  esac
done
echo "== all steps ok ($(date +%T))"
