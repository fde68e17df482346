set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sensitivity.py tests/test_gpu_cat.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6p_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6p_tests.txt; exit 1; }
tail -1 gpurun_out/r6p_tests.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6p_cat_prof -o cat -- python3 bench.py --task cat --no-cpu-baseline --steps 200 > gpurun_out/r6p_cat_bench.json 2> gpurun_out/r6p_cat_prof.log || { echo "rocprof failed"; tail -20 gpurun_out/r6p_cat_prof.log; exit 1; }
tail -1 gpurun_out/r6p_cat_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('CAT', d['value']/1e6, d['ms_per_step']*1e3)"
find gpurun_out/r6p_cat_prof -name "*kernel_stats.csv" | head -1 | xargs cat | head -12
