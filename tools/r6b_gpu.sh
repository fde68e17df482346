set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_iter.sh r6b || exit 1
bash tools/ab_run.sh r6b 2 - epb16h_half epb16h_halfx
