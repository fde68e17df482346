mkdir -p gpurun_out
for t in phase no_early no_store phase; do
  timeout -k 10 200 python -u tools/phase_profile.py --tag $t > gpurun_out/r4f_$t.json 2>gpurun_out/r4f_$t.err || { echo "fail $t"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r4f_$t.json').read().strip().splitlines()[-1]); r=d['cycles_per_wave_per_env_step']
print('$t', r.get('wave_realtime_us_median'))
for k,v in r.get('per_xcc_us_median',{}).items(): print(' ', k, {a: v[a] for a in ('physics','sensor..reset','store issue','store completion','end','barrier R2 wait')})"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py -m gpu -v -s --timeout 500 --timeout-method thread > gpurun_out/r4f_rollout_tests.txt 2>&1 || { echo "rollout tests failed"; tail -30 gpurun_out/r4f_rollout_tests.txt; exit 1; }
grep -E "PASS|FAIL|C4 rehearsal" gpurun_out/r4f_rollout_tests.txt | cut -c1-300
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 300 python -u bench.py --rollout on --force-collective --no-cpu-baseline --steps 240 --warmup 48 > gpurun_out/r4f_rccl_rollout.json 2> gpurun_out/r4f_rccl_rollout.err || { echo "rccl bench failed"; tail -20 gpurun_out/r4f_rccl_rollout.err; exit 1; }
tail -1 gpurun_out/r4f_rccl_rollout.json | cut -c1-600
