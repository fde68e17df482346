#!/bin/bash
# A/B on one GPU box: the default bench line with environment variable VAR=A and VAR=B, alternating, 2 runs each.
# Usage: bash tools/ab_env.sh <tag> <VAR> <A> <B> [bench args...]
set -o pipefail
tag=$1 var=$2 va=$3 vb=$4
shift 4
for r in 1 2; do
  for v in "$va" "$vb"; do
    export "$var=$v"
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1000 "$@" > gpurun_out/${tag}_$v$r.json 2>&1 || { echo "bench $var=$v failed"; tail -5 gpurun_out/${tag}_$v$r.json; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${tag}_$v$r.json').read().strip().splitlines()[-1]); print('$var=$v', $r, round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2), 'second', round(d['roofline']['secondary']['kernel_ms_avg']*1e3,2))"
  done
done
