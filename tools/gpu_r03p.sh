mkdir -p gpurun_out/r03p && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03p/t.log 2>&1
rc=$?; tail -2 gpurun_out/r03p/t.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  CBG_AOS=$v timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/r03p/b$v.log 2>&1 || exit 13
  python3 -c "import json;d=json.loads(open('gpurun_out/r03p/b$v.log').read().splitlines()[-1]);print('AOS=$v', round(d['ms_per_step'],2), d['phases_ms']['heavy_ms'], d['phases_ms']['numeric_ms'], round(d['roofline']['frac'],4), d['verified']['bit_exact'])"
done
CBG_AOS=1 timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 --scale 21 > gpurun_out/r03p/s21.log 2>&1 || exit 4
python3 -c "import json;d=json.loads(open('gpurun_out/r03p/s21.log').read().splitlines()[-1]);print('s21 AOS', round(d['ms_per_step'],2), d['phases_ms'], round(d['roofline']['frac'],4))"
