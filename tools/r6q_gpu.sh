set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cat.py tests/test_gpu_fused_obs.py tests/test_gpu_golden_terms.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r6q_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6q_tests.txt; exit 1; }
tail -1 gpurun_out/r6q_tests.txt
for r in 1 2; do
  timeout -k 10 200 python3 -u bench.py --task cat --no-cpu-baseline --steps 1000 > gpurun_out/r6q_cat_new$r.json 2>/dev/null || { echo "cat bench failed"; exit 1; }
  H12ENV_LIB=$PWD/tools/_variants/lib_r6lds.so timeout -k 10 200 python3 -u bench.py --task cat --no-cpu-baseline --steps 1000 > gpurun_out/r6q_cat_old$r.json 2>/dev/null || { echo "cat bench old failed"; exit 1; }
  for v in new old; do tail -1 gpurun_out/r6q_cat_$v$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cat $v', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), 'step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"; done
done
