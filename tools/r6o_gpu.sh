set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6o_gputest.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r6o_gputest.txt; exit 1; }
tail -1 gpurun_out/r6o_gputest.txt
bash tools/ab_run.sh r6o 3 - r6lds
H12_PHASE_LIGHT=1 H12_WAVE_DUMP=gpurun_out/r6o_waves.npy timeout -k 10 200 python3 -u tools/phase_profile.py --tag light > gpurun_out/r6o_light.json 2>/dev/null || { echo "light failed"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6o_light.json'))['cycles_per_wave_per_env_step']; print(json.dumps(d.get('block_tail')))"


