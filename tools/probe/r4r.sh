# -fassociative-math variant: A/B bench against the product, then the whole GPU suite on it
set -o pipefail
mkdir -p gpurun_out
V=$PWD/h1v2-isaac_amd/h12env/libh12env_assoc.so
for r in 1 2 3; do
  for v in plain assoc; do
    unset H12ENV_LIB
    [ $v = assoc ] && export H12ENV_LIB=$V
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 1000 > gpurun_out/r4r_$v$r.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r4r_$v$r.json').read().strip().splitlines()[-1]); print('$v run $r', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
  done
done
export H12ENV_LIB=$V
H12_FORCED_LOG=gpurun_out/r4r_forced.log timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -rf > gpurun_out/r4r_gputest.txt 2>&1
echo "suite rc=$?"; tail -15 gpurun_out/r4r_gputest.txt | cut -c1-300
