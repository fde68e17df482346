# round 5: the whole -m gpu suite (incl. the sole-contact gates), then the default bench line
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_gputest.txt 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/${tag}_gputest.txt | head -20; tail -5 gpurun_out/${tag}_gputest.txt; exit 1; }
tail -1 gpurun_out/${tag}_gputest.txt
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 1000 > gpurun_out/${tag}_bench.json 2>&1 || { echo bench failed; tail -5 gpurun_out/${tag}_bench.json; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_bench.json').read().strip().splitlines()[-1]); print('BENCH', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
