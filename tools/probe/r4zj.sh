# light stamps with the post-rewards / post-L marks (physics wave phases, waves with / without a resetting env), then
# the round's task lines
set -o pipefail
mkdir -p gpurun_out
H12_PHASE_LIGHT=1 timeout -k 10 200 python3 -u tools/phase_profile.py --tag light > gpurun_out/r4zj_light.json 2>/dev/null || { echo "light failed"; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4zj_light.json').read().strip().splitlines()[-1]); r=d['cycles_per_wave_per_env_step']; print(json.dumps(r.get('light_phases_us_median'))); print(r['wave_realtime_us_median'])"
bash tools/probe/r4zi.sh
