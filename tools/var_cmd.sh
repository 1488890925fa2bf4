# dev helper: benchmark tuning variants (tools/var/*) against the product library on one GPU
set -u
mkdir -p gpurun_out/var
timeout -k 10 400 python -u tools/var_bench.py "$@" -- --steps 3 --warmup 1 --no-cpu > gpurun_out/var/var.log 2>&1
rc=$?; cat gpurun_out/var/var.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/var/base.log 2>&1 || exit 3
tail -1 gpurun_out/var/base.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('base', j['ms_per_step'], j['config']['nnz_C'], j['phases_ms'])"
if [ -n "${VAR_TEST:-}" ]; then
  CBG_LIB_PATH=$PWD/tools/var/$VAR_TEST/libcbgpu.so timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/var/test.log 2>&1; tail -2 gpurun_out/var/test.log
fi
