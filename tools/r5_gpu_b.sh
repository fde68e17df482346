# round 5: light-stamp profile (barrier waits per wave role) of the in-tree kernel, then an A/B against other libraries
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5}
shift
H12_PHASE_LIGHT=1 timeout -k 10 200 python3 -u tools/phase_profile.py --tag light > gpurun_out/${tag}_light.json 2>/dev/null || { echo "light failed"; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_light.json').read().strip().splitlines()[-1]); r=d['cycles_per_wave_per_env_step']; print(json.dumps(r.get('barrier_wait_us_per_launch_median'))); print(json.dumps(r.get('light_phases_us_median'))); print(r['wave_realtime_us_median'])"
bash tools/ab_run.sh ${tag}_ab 2 - "$@"
