#!/bin/bash
# A/B of the main library against tools/var/prev (the previous commit, `make var VAR=prev` from its sources): GPU parity
# of the heavy path on main, s20 bench x2, s22 rank shares 0 and 4, rocprofv3 kernel stats of main at s20.  usage: [TESTS=tests] ab_prev.sh <tag>
set -u
O=gpurun_out/${1:?tag}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest ${TESTS:-tests/test_spgemm_gpu.py tests/test_fullsize_gpu.py} -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -15 $O/tests.log; exit 11; }
tail -2 $O/tests.log
for r in 1 2; do
timeout -k 10 600 python3 -u tools/var_bench.py main prev -- --no-cpu --steps 10 --scale 20 > $O/var_s20_$r.log 2>&1 || { tail -5 $O/var_s20_$r.log; exit 12; }
cut -c1-300 $O/var_s20_$r.log
done
timeout -k 10 600 python3 -u tools/var_bench.py main prev -- --rank-share 0,4 --gpus-virtual 8 --scale 22 --no-cpu > $O/var_share22.log 2>&1 || { tail -5 $O/var_share22.log; exit 13; }
cut -c1-300 $O/var_share22.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 14; }
tail -1 $O/prof.log | cut -c1-300
