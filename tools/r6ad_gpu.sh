set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r6ad_tests.txt 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r6ad_tests.txt; exit 1; }
tail -1 gpurun_out/r6ad_tests.txt
for task in rsl c5 rough; do
  timeout -k 10 200 python3 -u bench.py --task $task --no-cpu-baseline --steps 1000 > gpurun_out/r6ad_$task.json 2>/dev/null || { echo "bench $task failed"; exit 1; }
  tail -1 gpurun_out/r6ad_$task.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$task', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), 'step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
done
