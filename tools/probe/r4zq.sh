# self-contact narrow phase: only the flagged groups' jobs, compacted over the candidate envs (new) vs the final build (base)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused_obs.py tests/test_gpu_edge.py tests/test_gpu_parity.py tests/test_gpu_selfcollision.py tests/test_gpu_longrun.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4zq_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4zq_tests.txt; exit 1; }
tail -2 gpurun_out/r4zq_tests.txt
for r in 1 2 3; do
  for v in new base; do
    unset H12ENV_LIB
    [ $v != new ] && export H12ENV_LIB=$PWD/tools/_variants/lib_$v.so
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 1000 > gpurun_out/r4zq_$v$r.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r4zq_$v$r.json').read().strip().splitlines()[-1]); print('$v run $r', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
  done
done
unset H12ENV_LIB
