#!/bin/bash
# A/B on one GPU box: the default bench line with each listed library variant (h1v2-isaac_amd/h12env/libh12env_<v>.so;
# "cur" = the in-tree libh12env.so), one run each, twice round.  Usage: bash tools/ab_libs.sh <tag> <v1> <v2> ...
set -o pipefail
tag=$1
shift
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = cur ]; then unset H12ENV_LIB; else export H12ENV_LIB=$PWD/h1v2-isaac_amd/h12env/libh12env_$v.so; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1000 > gpurun_out/${tag}_$v$r.json 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/${tag}_$v$r.json; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${tag}_$v$r.json').read().strip().splitlines()[-1]); print('$v', $r, round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2), 'second', round(d['roofline']['secondary']['kernel_ms_avg']*1e3,2))"
  done
done
