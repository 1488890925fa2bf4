# A/B of the overlapped decode in the RCCL rehearsal (2 and 8 ranks on one GPU) and the s21 N=2 rank share
set -u
mkdir -p gpurun_out/r06f
export TMPDIR=/tmp
for ov in 1 0; do
  for n in 2 8; do
    CBG_FIBER_DECODE_OVERLAP=$ov CBG_DIST_BACKEND=rccl-net timeout -k 10 300 python3 bench.py --gpus $n --steps 3 --warmup 1 --scale 18 --no-cpu \
      > gpurun_out/r06f/launch_n${n}_ov$ov.json 2> gpurun_out/r06f/launch_n${n}_ov$ov.err || { tail -5 gpurun_out/r06f/launch_n${n}_ov$ov.err; exit 11; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06f/launch_n${n}_ov$ov.json').read().strip().splitlines()[-1]); p=d['rank0_phases_per_step']; print('ov=$ov n=$n', round(d['ms_per_step'],2), {k: round(p[k],2) for k in ('local_ms','merge_ms','fiber_ms','fiber_xfer_ms')})"
  done
done
