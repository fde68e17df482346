# slack of the self-contact / helper waves in the R1 -> R2 window (300 dependent VALU per inner step, tools/variant.py)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in plain self_r2slack300 helper_r2slack300; do
    unset H12ENV_LIB
    [ $v != plain ] && export H12ENV_LIB=$PWD/tools/_variants/lib_$v.so
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 1000 > gpurun_out/r4zo_$v$r.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r4zo_$v$r.json').read().strip().splitlines()[-1]); print('$v run $r', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
  done
done
