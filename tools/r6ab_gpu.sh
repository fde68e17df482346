set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rough.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r6ab_tests.txt 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r6ab_tests.txt; exit 1; }
tail -1 gpurun_out/r6ab_tests.txt
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export H12ENV_LIB=$PWD/tools/_variants/lib_r6head.so; else unset H12ENV_LIB; fi
    timeout -k 10 200 python3 -u bench.py --task rough --no-cpu-baseline --steps 1000 > gpurun_out/r6ab_rough_$v$r.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    tail -1 gpurun_out/r6ab_rough_$v$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rough $v', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), 'step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2), 'obs', d['roofline'].get('second_kernel', {}).get('kernel_ms_avg') if isinstance(d['roofline'].get('second_kernel'), dict) else '')"
  done
done
