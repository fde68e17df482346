# round 5: GPU suite, then the light-stamp profile and an A/B against the given variant libraries
set -o pipefail
tag=${1:-r5}
shift
bash tools/r5_gpu_a.sh $tag || exit 1
bash tools/r5_gpu_b.sh $tag "$@"
