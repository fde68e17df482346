set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r6w_cat -o cat -- python3 bench.py --task cat --no-cpu-baseline --steps 200 > gpurun_out/r6w_cat.json 2> gpurun_out/r6w_cat.err || { echo "cat prof failed"; tail -20 gpurun_out/r6w_cat.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r6w_rough -o rough -- python3 bench.py --task rough --no-cpu-baseline --steps 200 > gpurun_out/r6w_rough.json 2> gpurun_out/r6w_rough.err || { echo "rough prof failed"; tail -20 gpurun_out/r6w_rough.err; exit 1; }
find gpurun_out/r6w_cat gpurun_out/r6w_rough -name "*stats*"
