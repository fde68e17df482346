#!/bin/bash
# A/B of step_kernel's per-XCD block weights (H12_XCD_WEIGHTS, csrc xcd_table) on one GPU box.
set -o pipefail
tag=${1:-xcd}
for r in 1 2; do
  for w in "1,1,1,1,1,1,1,1" "2,2,1,1,1,1,2,2" "3,3,1,1,1,1,3,3" "4,4,1,1,1,1,4,4"; do
    H12_XCD_WEIGHTS=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1000 > gpurun_out/${tag}.json 2>&1 || { echo "bench $w failed"; tail -5 gpurun_out/${tag}.json; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/${tag}.json').read().strip().splitlines()[-1]); print('$w', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2), 'exact', d['replay_bit_exact'])"
  done
done
