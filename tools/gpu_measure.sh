#!/bin/bash
# GPU box: the round's measurement set after a green suite -- rocprofv3 stats + PMC passes (tools/profile.sh), the
# task / mode variants of bench.py, and the MuJoCo-mode contact statistic.  Every step under its own time limit;
# stops at the first failure.  Usage: bash tools/gpu_measure.sh <tag>
set -o pipefail
tag=${1:-r3}
o=gpurun_out
bash tools/profile.sh $tag > $o/${tag}_profile.log 2>&1 || { echo "profile failed"; tail -20 $o/${tag}_profile.log; exit 1; }
echo "profile ok"
for t in rough c5 rsl cat; do
  timeout -k 10 300 python -u bench.py --task $t --no-cpu-baseline > $o/${tag}_bench_$t.json 2> $o/${tag}_bench_$t.err || { echo "bench $t failed"; tail -20 $o/${tag}_bench_$t.err; exit 1; }
  echo "bench $t ok"
done
timeout -k 10 300 python -u bench.py --rollout on --no-cpu-baseline > $o/${tag}_bench_rollout.json 2> $o/${tag}_bench_rollout.err || { echo "bench rollout failed"; exit 1; }
echo "bench rollout ok"
timeout -k 10 300 python -u bench.py --rollout on --rollout-decode --no-cpu-baseline > $o/${tag}_bench_rollout_decode.json 2> $o/${tag}_bench_rollout_decode.err || { echo "bench rollout decode failed"; exit 1; }
echo "bench rollout decode ok"
timeout -k 10 600 python -u bench.py --mode train --no-cpu-baseline > $o/${tag}_bench_train.json 2> $o/${tag}_bench_train.err || { echo "bench train failed"; tail -20 $o/${tag}_bench_train.err; exit 1; }
echo "bench train ok"
timeout -k 10 600 python -u tools/mujoco_contact_stats.py --out $o/${tag}_mujoco_contact.json > $o/${tag}_mujoco_contact.log 2>&1 || { echo "mujoco stats failed"; tail -20 $o/${tag}_mujoco_contact.log; exit 1; }
echo "mujoco stats ok"
