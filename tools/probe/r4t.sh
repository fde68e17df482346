set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --mode train --iterations 10 --no-cpu-baseline > gpurun_out/r4t_base_$r.json 2>/dev/null && tail -1 gpurun_out/r4t_base_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', round(d['value']/1e6,3), 'M learn', round(d['learning_s_per_iter']*1e3,2))"
  TORCH_BLAS_PREFER_HIPBLASLT=0 timeout -k 10 300 python3 -u bench.py --mode train --iterations 10 --no-cpu-baseline > gpurun_out/r4t_rocblas_$r.json 2>gpurun_out/r4t_rocblas_$r.err && tail -1 gpurun_out/r4t_rocblas_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rocblas', round(d['value']/1e6,3), 'M learn', round(d['learning_s_per_iter']*1e3,2))"
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=/tmp/tunableop_%d.csv timeout -k 10 400 python3 -u bench.py --mode train --iterations 10 --no-cpu-baseline > gpurun_out/r4t_tunable_$r.json 2>gpurun_out/r4t_tunable_$r.err && tail -1 gpurun_out/r4t_tunable_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tunableop', round(d['value']/1e6,3), 'M learn', round(d['learning_s_per_iter']*1e3,2))" || { echo "tunable failed"; tail -5 gpurun_out/r4t_tunable_$r.err; }
done
