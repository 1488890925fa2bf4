#!/bin/bash
# r04a: kernel parity after the ticketed heavy grids, the bench line with the reference's own CPU baseline,
# the RCCL-footprint co-residency probe (ticketed vs static heavy grid, with/without a CU reservation), and the
# rank shares of the 8-GPU 2x2x2 layout at scale 22 on this one GPU.
set -u
OUT=gpurun_out/r04a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log | cut -c1-800; exit 13; }
tail -1 $OUT/bench.log | cut -c1-2500
for v in "dyn:" "static:tools/var/static/libcbgpu.so" ; do
  name=${v%%:*}; lib=${v#*:}
  extra=""; [ -n "$lib" ] && extra="--lib $lib"
  timeout -k 10 180 python -u tools/coresidency_probe.py --tag $name $extra >> $OUT/probe.jsonl 2>> $OUT/probe.err || { echo "probe $name failed"; tail -5 $OUT/probe.err; exit 4; }
done
CBG_HEAVY_RESERVE_CU=16 timeout -k 10 180 python -u tools/coresidency_probe.py --tag dyn_reserve16 >> $OUT/probe.jsonl 2>> $OUT/probe.err || { echo "probe reserve failed"; exit 4; }
cut -c1-900 $OUT/probe.jsonl
timeout -k 10 900 python -u bench.py --rank-share all --gpus-virtual 8 --scale 22 > $OUT/rank_share_s22.jsonl 2> $OUT/rank_share.err
rc=$?; cut -c1-700 $OUT/rank_share_s22.jsonl; tail -3 $OUT/rank_share.err; exit $rc
