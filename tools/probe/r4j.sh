set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/probe/reduce_bench.py > gpurun_out/r4j_reduce.txt 2>&1 || echo "reduce bench failed"
for r in 1 2 3; do
  for k in 0 1; do
    HIP_FORCE_DEV_KERNARG=$k timeout -k 10 200 python3 -u tools/phase_profile.py --tag phase > gpurun_out/r4j_kernarg${k}_$r.json 2>/dev/null || { echo "phase failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r4j_kernarg${k}_$r.json').read().strip().splitlines()[-1]); r=d['cycles_per_wave_per_env_step']['per_xcc_us_median']
print('devkernarg=$k run $r', ' '.join(f\"{x[3:]}:{v['physics']:.1f}/{v['sensor..reset']:.1f}/{v['end']:.1f}\" for x,v in r.items()))"
  done
done
