set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probe/hw_bias > gpurun_out/r6f_hw_bias.txt 2>&1 || { echo "hw_bias failed"; exit 1; }
cat gpurun_out/r6f_hw_bias.txt
timeout -k 10 600 python -u tools/bias_probe.py --runs flight,lying,stance,single_stance,slip --json gpurun_out/r6f_bias_probe.json > gpurun_out/r6f_bias_probe.txt 2>&1 || { echo "bias probe failed"; tail -20 gpurun_out/r6f_bias_probe.txt; exit 1; }
cat gpurun_out/r6f_bias_probe.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6f_gputest.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r6f_gputest.txt; exit 1; }
tail -1 gpurun_out/r6f_gputest.txt
bash tools/ab_run.sh r6f 2 - r6prev
