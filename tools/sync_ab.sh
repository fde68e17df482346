#!/bin/bash
# GPU box: the driver's bench command (--steps 20 --warmup 5) under the HIP runtime's default host wait and under
# longer active (spinning) waits / device-memory kernel arguments, interleaved, 3 runs each.
# Usage: bash tools/sync_ab.sh <tag>
set -o pipefail
tag=${1:-sync}
o=gpurun_out/$tag
mkdir -p $o
for r in 1 2 3; do
  for v in default spin devkarg; do
    case $v in
      default) env_set="" ;;
      spin) env_set="ROC_ACTIVE_WAIT_TIMEOUT=100000" ;;
      devkarg) env_set="HIP_FORCE_DEV_KERNARG=1" ;;
    esac
    env $env_set timeout -k 10 240 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $o/${v}_$r.json 2> $o/${v}_$r.err || { echo "bench $v $r failed"; tail -5 $o/${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$o/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, round(d['value']/1e6, 2), 'M', round(d['ms_per_step']*1e3, 2), 'us/step')"
  done
done
