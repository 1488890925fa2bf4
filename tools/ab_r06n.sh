# A/B: adaptive unit span (main library) vs the fixed span cap (tools/var/noadapt), s20 / s22 rank shares / s21
set -u
mkdir -p gpurun_out/r06n
export TMPDIR=/tmp
for r in 1 2; do
timeout -k 10 600 python3 -u tools/var_bench.py main hm3 hm2 -- --no-cpu --steps 10 --scale 20 > gpurun_out/r06n/var_s20_$r.log 2>&1 || { tail -5 gpurun_out/r06n/var_s20_$r.log; exit 11; }
cut -c1-300 gpurun_out/r06n/var_s20_$r.log
done
timeout -k 10 600 python3 -u tools/var_bench.py main hm3 hm2 -- --rank-share 0,4 --gpus-virtual 8 --scale 22 --no-cpu > gpurun_out/r06n/var_share22.log 2>&1 || { tail -5 gpurun_out/r06n/var_share22.log; exit 12; }
cat gpurun_out/r06n/var_share22.log | cut -c1-300
timeout -k 10 600 python3 -u tools/var_bench.py main hm3 hm2 -- --no-cpu --steps 3 --scale 21 > gpurun_out/r06n/var_s21.log 2>&1 || { tail -5 gpurun_out/r06n/var_s21.log; exit 13; }
cut -c1-300 gpurun_out/r06n/var_s21.log
