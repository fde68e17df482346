# round 5: light-stamp profile + rocprofv3 stats / PMC passes (tools/profile.sh) of the in-tree kernel
set -o pipefail
tag=${1:-r5}
H12_PHASE_LIGHT=1 timeout -k 10 200 python3 -u tools/phase_profile.py --tag light > gpurun_out/${tag}_light.json 2>/dev/null || { echo "light failed"; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_light.json').read().strip().splitlines()[-1]); r=d['cycles_per_wave_per_env_step']; print(json.dumps(r.get('barrier_wait_us_per_launch_median'))); print(json.dumps(r.get('light_phases_us_median'))); print(r['wave_realtime_us_median'])"
bash tools/profile.sh $tag && grep -E "step_kernel" profiles/${tag}_kernel_stats.csv | head -3
