set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cat_inline.py tests/test_gpu_cat.py tests/test_gpu_fused_obs.py tests/test_gpu_golden_terms.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r6x_tests.txt 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r6x_tests.txt; exit 1; }
tail -1 gpurun_out/r6x_tests.txt
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export H12ENV_LIB=$PWD/tools/_variants/lib_r6pad.so; else unset H12ENV_LIB; fi
    for task in cat flat; do
      timeout -k 10 200 python3 -u bench.py --task $task --no-cpu-baseline --steps 1000 > gpurun_out/r6x_${task}_$v$r.json 2>/dev/null || { echo "bench $task $v failed"; exit 1; }
      tail -1 gpurun_out/r6x_${task}_$v$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$task $v', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), 'step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
    done
  done
done
