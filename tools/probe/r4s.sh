set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for k in 16 8 32 64; do
    H12_SPLIT_K=$k timeout -k 10 300 python3 -u bench.py --mode train --iterations 10 --no-cpu-baseline > gpurun_out/r4s_k${k}_$r.json 2>/dev/null || { echo "train k=$k failed"; exit 1; }
    tail -1 gpurun_out/r4s_k${k}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('split_k=$k', round(d['value']/1e6,3), 'M', 'learn', round(d['learning_s_per_iter']*1e3,2), 'ms')"
  done
done
