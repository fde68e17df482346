set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r6ao_tests.txt 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r6ao_tests.txt; exit 1; }
tail -1 gpurun_out/r6ao_tests.txt
for t in rsl cat flat; do timeout -k 10 200 python -u tools/probe/determinism.py $t 8192 300 2>&1 | grep -v amdgpu.ids || exit 1; done
bash tools/ab_run.sh r6ao 3 - r6fin
