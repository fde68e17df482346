# learner A/B (twin actor+critic vs separate), the icache counter passes, the learner kernel breakdown
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for tw in 1 0; do
    H12_TWIN=$tw timeout -k 10 300 python3 -u bench.py --mode train --iterations 10 --no-cpu-baseline > gpurun_out/r4i_train_twin${tw}_$r.json 2>gpurun_out/r4i_train_twin${tw}_$r.err || { echo "train twin=$tw failed"; tail -5 gpurun_out/r4i_train_twin${tw}_$r.err; exit 1; }
    tail -1 gpurun_out/r4i_train_twin${tw}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('twin=$tw', round(d['value']/1e6,3), 'M', 'learn', round(d['learning_s_per_iter']*1e3,2), 'ms', 'collect', round(d['collection_s_per_iter']*1e3,2), 'ms')"
  done
done
bash tools/probe/r4h.sh
