set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in new cat_fold_after_f cat_no_nmrows; do
    if [ $v = new ]; then unset H12ENV_LIB; else export H12ENV_LIB=$PWD/tools/_variants/lib_$v.so; fi
    timeout -k 10 200 python3 -u bench.py --task cat --no-cpu-baseline --steps 1000 > gpurun_out/r6z_cat_$v$r.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    tail -1 gpurun_out/r6z_cat_$v$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cat $v', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), 'step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
  done
done
