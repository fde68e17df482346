set -o pipefail
mkdir -p gpurun_out
for v in light no_torso no_drain; do
  H12_PHASE_LIGHT=1 H12_WAVE_DUMP=gpurun_out/r6m_${v}_waves.npy timeout -k 10 200 python3 -u tools/phase_profile.py --tag $v > gpurun_out/r6m_${v}.json 2>/dev/null || { echo "light $v failed"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r6m_${v}.json'))['cycles_per_wave_per_env_step']; b=d.get('block_tail'); print('$v', b['physics_loop_us_p50_p95_max'], b['per_launch_max_minus_median_us'])"
done
