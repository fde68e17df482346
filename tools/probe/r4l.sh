# A/B: device-resident KParams (in-tree lib) vs HEAD~ build (libh12env_base.so), default kernarg placement, and the
# base build with HIP_FORCE_DEV_KERNARG=1; then the GPU suite on the new lib
set -o pipefail
mkdir -p gpurun_out
B=$PWD/h1v2-isaac_amd/h12env/libh12env_base.so
for r in 1 2 3; do
  for v in new base basedev; do
    unset H12ENV_LIB HIP_FORCE_DEV_KERNARG
    [ $v = base ] && export H12ENV_LIB=$B
    [ $v = basedev ] && export H12ENV_LIB=$B HIP_FORCE_DEV_KERNARG=1
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 1000 > gpurun_out/r4l_$v$r.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r4l_$v$r.json').read().strip().splitlines()[-1]); print('$v run $r', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
  done
done
unset H12ENV_LIB HIP_FORCE_DEV_KERNARG
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r4l_drv.json 2>/dev/null && python3 -c "import json; d=json.loads(open('gpurun_out/r4l_drv.json').read().strip().splitlines()[-1]); print('driver cmd new', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
H12_FORCED_LOG=gpurun_out/r4l_forced.log timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4l_gputest.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r4l_gputest.txt; exit 1; }
tail -1 gpurun_out/r4l_gputest.txt
