set -o pipefail
mkdir -p gpurun_out
for v in new acc_rsq acc_rcp acc_sqrt acc_pre acc_all; do
  if [ "$v" = new ]; then unset H12ENV_LIB; else export H12ENV_LIB=$PWD/tools/_variants/lib_$v.so; fi
  echo "== $v"
  timeout -k 10 300 python -u tools/bias_probe.py --runs stance,lying --json gpurun_out/r6h_bias_$v.json > gpurun_out/r6h_bias_$v.txt 2>&1 || { echo "bias probe $v failed"; tail -20 gpurun_out/r6h_bias_$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r6h_bias_$v.txt
done
