set -o pipefail
mkdir -p gpurun_out
for t in rsl cat rough c5; do
  timeout -k 10 200 python3 -u bench.py --task $t --no-cpu-baseline --steps 1000 > gpurun_out/r4zp_$t.json 2>/dev/null || { echo "bench $t failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r4zp_$t.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$t', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step env', round(r['kernel_ms_avg']*1e3,2), 'second', round(r['secondary']['kernel_ms_avg']*1e3,2))"
done
timeout -k 10 200 python3 -u bench.py --rollout on --no-cpu-baseline --steps 1000 > gpurun_out/r4zp_rollout.json 2>/dev/null && python3 -c "import json; d=json.loads(open('gpurun_out/r4zp_rollout.json').read().strip().splitlines()[-1]); print('rollout on', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2))"
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r4zp_drv.json 2>/dev/null && python3 -c "import json; d=json.loads(open('gpurun_out/r4zp_drv.json').read().strip().splitlines()[-1]); print('driver cmd', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2))"
timeout -k 10 400 python3 -u bench.py --mode train --iterations 10 --no-cpu-baseline > gpurun_out/r4zp_train.json 2>/dev/null && python3 -c "import json; d=json.loads(open('gpurun_out/r4zp_train.json').read().strip().splitlines()[-1]); print('train', round(d['value']/1e6,3), 'M learn', round(d['learning_s_per_iter']*1e3,2), 'collect', round(d['collection_s_per_iter']*1e3,2))"
