set -u
mkdir -p gpurun_out/ab1
export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/var_bench.py nostage stage nostage stage -- --no-cpu --steps 5 > gpurun_out/ab1/g500seed.log 2>&1; echo rc=$?; cat gpurun_out/ab1/g500seed.log | cut -c1-400
timeout -k 10 600 python3 -u tools/var_bench.py nostage stage -- --no-cpu --steps 5 --seed 1 > gpurun_out/ab1/seed1.log 2>&1; echo rc=$?; cat gpurun_out/ab1/seed1.log | cut -c1-400
