# placement of the start-state reload (st_reload at the integration, _pair before the base pair sum, _p3 before pass 3)
set -o pipefail
mkdir -p gpurun_out
export H12ENV_LIB=$PWD/tools/_variants/lib_st_reload_p3.so
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused_obs.py tests/test_gpu_edge.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r4zf_tests.txt 2>&1 || { echo "variant tests failed"; tail -30 gpurun_out/r4zf_tests.txt; exit 1; }
tail -1 gpurun_out/r4zf_tests.txt
for r in 1 2 3; do
  for v in prod st_reload st_reload_pair st_reload_p3; do
    unset H12ENV_LIB
    [ $v != prod ] && export H12ENV_LIB=$PWD/tools/_variants/lib_$v.so
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 1000 > gpurun_out/r4zf_$v$r.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r4zf_$v$r.json').read().strip().splitlines()[-1]); print('$v run $r', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
  done
done
