set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for tu in 1 0; do
    H12_TUNABLEOP=$tu timeout -k 10 400 python3 -u bench.py --mode train --iterations 10 --no-cpu-baseline > gpurun_out/r4u_tune${tu}_$r.json 2>gpurun_out/r4u_tune${tu}_$r.err || { echo "train tune=$tu failed"; tail -5 gpurun_out/r4u_tune${tu}_$r.err; exit 1; }
    tail -1 gpurun_out/r4u_tune${tu}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tunableop=$tu', round(d['value']/1e6,3), 'M learn', round(d['learning_s_per_iter']*1e3,2), 'collect', round(d['collection_s_per_iter']*1e3,2))"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_deploy.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r4u_train_tests.txt 2>&1 || { echo "train tests failed"; tail -30 gpurun_out/r4u_train_tests.txt; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r4u_train_tests.txt | cut -c1-150; ls *.csv 2>/dev/null | head
