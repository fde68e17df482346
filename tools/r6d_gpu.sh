set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probe/hw_bias > gpurun_out/r6d_hw_bias.txt 2>&1 || { echo "hw_bias failed"; exit 1; }
cat gpurun_out/r6d_hw_bias.txt
bash tools/ab_run.sh r6d 2 - self_noatomic
