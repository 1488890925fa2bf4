set -u
mkdir -p gpurun_out/diag1
timeout -k 10 300 python3 -u tools/diag_s20.py 20 6 gpurun_out/diag1/new.json > gpurun_out/diag1/new.log 2>&1; echo "new rc=$?"
tail -c 3000 gpurun_out/diag1/new.log
CBG_LIB_PATH=$PWD/tools/var/old/libcbgpu.so timeout -k 10 300 python3 -u tools/diag_s20.py 20 6 gpurun_out/diag1/old.json > gpurun_out/diag1/old.log 2>&1; echo "old rc=$?"
head -c 1500 gpurun_out/diag1/old.log
CBG_LIB_PATH=$PWD/tools/var/norank/libcbgpu.so timeout -k 10 300 python3 -u tools/diag_s20.py 20 6 gpurun_out/diag1/norank.json > gpurun_out/diag1/norank.log 2>&1; echo "norank rc=$?"
head -c 1500 gpurun_out/diag1/norank.log
