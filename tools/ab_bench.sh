#!/bin/bash
# A/B on one GPU box: the default bench line with the in-tree libh12env.so and with h12env/libh12env_base.so
# (a baseline build), alternating, 2 runs each.  Usage: bash tools/ab_bench.sh <tag>
set -o pipefail
tag=${1:-ab}
for r in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export H12ENV_LIB=$PWD/h1v2-isaac_amd/h12env/libh12env_base.so; else unset H12ENV_LIB; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1000 > gpurun_out/${tag}_$v$r.json 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/${tag}_$v$r.json; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${tag}_$v$r.json').read().strip().splitlines()[-1]); print('$v$r', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2), 'obs', round(d['roofline']['secondary']['kernel_ms_avg']*1e3,2))"
  done
done
