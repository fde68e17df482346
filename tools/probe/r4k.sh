# product bench A/B: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the runtime default
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for k in d 1; do
    if [ $k = 1 ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 1000 > gpurun_out/r4k_$k$r.json 2>/dev/null || { echo "bench failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r4k_$k$r.json').read().strip().splitlines()[-1]); print('devkernarg=$k run $r', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
  done
done
unset HIP_FORCE_DEV_KERNARG
for k in d 1; do
  if [ $k = 1 ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r4k_drv_$k.json 2>/dev/null || { echo "bench failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r4k_drv_$k.json').read().strip().splitlines()[-1]); print('driver cmd devkernarg=$k', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
done
