set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3 4; do
  timeout -k 10 200 python3 -u tools/phase_profile.py --tag light > gpurun_out/r4m_light_$r.json 2>/dev/null || { echo "phase failed"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r4m_light_$r.json').read().strip().splitlines()[-1]); r=d['cycles_per_wave_per_env_step']
print('light run $r', r['wave_realtime_us_median'])
for x,v in r['per_xcc_us_median'].items(): print('   ', x, {k: v[k] for k in ('physics','sensor..reset','frame+F wait','store issue','store completion','end')})"
done
