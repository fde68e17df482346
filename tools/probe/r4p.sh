set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in plain scan_nogather; do
    for t in rough c5; do
      unset H12ENV_LIB
      [ $v != plain ] && export H12ENV_LIB=$PWD/tools/_variants/lib_$v.so
      timeout -k 10 200 python3 -u bench.py --task $t --no-cpu-baseline --steps 500 > gpurun_out/r4p_${t}_$v$r.json 2>/dev/null || { echo "bench $t $v failed"; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/r4p_${t}_$v$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$t $v run $r', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step env', round(r['kernel_ms_avg']*1e3,2), 'obs', round(r['secondary']['kernel_ms_avg']*1e3,2))"
    done
  done
done
