set -u
mkdir -p gpurun_out/r06d
export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/var_bench.py base h12 p19 -- --no-cpu --steps 5 --scale 20 > gpurun_out/r06d/var_s20.log 2>&1 || { tail -5 gpurun_out/r06d/var_s20.log; exit 11; }
cat gpurun_out/r06d/var_s20.log | cut -c1-400
timeout -k 10 600 python3 -u tools/var_bench.py base h12 p19 -- --rank-share 0,4 --gpus-virtual 8 --scale 22 --no-cpu > gpurun_out/r06d/var_share22.log 2>&1 || { tail -5 gpurun_out/r06d/var_share22.log; exit 12; }
cat gpurun_out/r06d/var_share22.log | cut -c1-400
timeout -k 10 600 python3 -u tools/var_bench.py base h12 p19 -- --no-cpu --steps 3 --scale 21 > gpurun_out/r06d/var_s21.log 2>&1 || { tail -5 gpurun_out/r06d/var_s21.log; exit 13; }
cat gpurun_out/r06d/var_s21.log | cut -c1-400
