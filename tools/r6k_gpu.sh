set -o pipefail
mkdir -p gpurun_out
echo "== product"
timeout -k 10 300 python -u -m pytest tests/test_gpu_rough.py -m gpu -q --timeout 200 --timeout-method thread -k "reset_and_steps" > gpurun_out/r6k_rough_new.txt 2>&1; tail -3 gpurun_out/r6k_rough_new.txt
echo "== torso_lane0"
H12ENV_LIB=$PWD/tools/_variants/lib_torso_lane0.so timeout -k 10 300 python -u -m pytest tests/test_gpu_rough.py -m gpu -q --timeout 200 --timeout-method thread -k "reset_and_steps" > gpurun_out/r6k_rough_lane0.txt 2>&1; tail -3 gpurun_out/r6k_rough_lane0.txt
echo "== r6trig (the last commit)"
H12ENV_LIB=$PWD/tools/_variants/lib_r6trig.so timeout -k 10 300 python -u -m pytest tests/test_gpu_rough.py -m gpu -q --timeout 200 --timeout-method thread -k "reset_and_steps" > gpurun_out/r6k_rough_trig.txt 2>&1; tail -3 gpurun_out/r6k_rough_trig.txt
