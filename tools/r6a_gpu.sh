set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_selfcollision.py tests/test_gpu_fused_obs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6a_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6a_tests.txt; exit 1; }
tail -1 gpurun_out/r6a_tests.txt
H12ENV_LIB=$PWD/tools/_variants/lib_epb16h.so timeout -k 10 400 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_fused_obs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6a_epb16h_tests.txt 2>&1 || { echo "epb16h tests failed"; tail -30 gpurun_out/r6a_epb16h_tests.txt; exit 1; }
tail -1 gpurun_out/r6a_epb16h_tests.txt
bash tools/ab_run.sh r6a 2 - epb16h chain_half epb16h_half
