#!/bin/bash
# One GPU-box pass for a round checkpoint: -m gpu tests, the default bench line, rocprofv3 stats + PMC.
# Usage (from the repo root, on the GPU box): bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-latest}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gputest_$TAG.txt; exit 1; }
tail -1 gpurun_out/gputest_$TAG.txt
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
bash tools/profile.sh "$TAG"
