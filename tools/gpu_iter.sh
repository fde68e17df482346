#!/bin/bash
# Quick GPU iteration: a named subset of -m gpu tests (default: all), then the default bench line.
# Usage (GPU box, repo root): bash tools/gpu_iter.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-iter}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/gputest_$TAG.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gputest_$TAG.txt; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gputest_$TAG.txt; exit 1; }
fi
tail -1 gpurun_out/gputest_$TAG.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value']/1e6, 'M', d['ms_per_step'], 'ms', 'step_kernel', d['roofline']['kernel_ms_avg'])"
