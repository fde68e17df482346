set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for f in 1 0; do
    H12_FUSED_MLP=$f timeout -k 10 300 python3 -u bench.py --mode train --iterations 10 --no-cpu-baseline > gpurun_out/r4n_train_fused${f}_$r.json 2>/dev/null || { echo "train fused=$f failed"; exit 1; }
    tail -1 gpurun_out/r4n_train_fused${f}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused_mlp=$f', round(d['value']/1e6,3), 'M', 'learn', round(d['learning_s_per_iter']*1e3,2), 'ms', 'collect', round(d['collection_s_per_iter']*1e3,2), 'ms')"
  done
done
H12_FUSED_MLP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4n_train_tests.txt 2>&1 || { echo "train tests failed"; tail -30 gpurun_out/r4n_train_tests.txt; exit 1; }
tail -1 gpurun_out/r4n_train_tests.txt
bash tools/probe/r4m.sh
