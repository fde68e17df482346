# CaT: compacted no_move rows (cat_reduce single-pass chunks, cat_prob one dependent load) -- tests, A/B, rocprof
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_cat.py tests/test_gpu_golden_terms.py tests/test_gpu_edge.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4zl_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4zl_tests.txt; exit 1; }
tail -1 gpurun_out/r4zl_tests.txt
for r in 1 2 3; do
  for v in new base; do
    unset H12ENV_LIB
    [ $v != new ] && export H12ENV_LIB=$PWD/tools/_variants/lib_$v.so
    timeout -k 10 200 python3 -u bench.py --task cat --no-cpu-baseline --steps 1000 > gpurun_out/r4zl_$v$r.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r4zl_$v$r.json').read().strip().splitlines()[-1]); print('cat $v run $r', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
  done
done
unset H12ENV_LIB
R=$PWD
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d /tmp/catprof -o run -- python3 $R/bench.py --task cat --steps 200 --warmup 20 --no-cpu-baseline --profile-only > $R/gpurun_out/r4zl_cat_prof.log 2>&1 && find /tmp/catprof -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r4zl_cat_kernel_stats.csv \;
cd $R && python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r4zl_cat_kernel_stats.csv')):
    if 'cat_' in r['Name'] or 'step_kernel' in r['Name']: print(r['Name'][:50], r['Calls'], r['AverageNs'])"
