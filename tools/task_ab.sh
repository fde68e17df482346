#!/bin/bash
# GPU box: bench lines of the given tasks for the in-tree library ("cur") and the listed variants
# (h1v2-isaac_amd/h12env/libh12env_<v>.so), interleaved, twice round.  Usage: bash tools/task_ab.sh <tag> "<tasks>" <v> ...
set -o pipefail
tag=$1; tasks=$2; shift 2
o=gpurun_out/$tag
mkdir -p $o
for r in 1 2; do
  for v in cur "$@"; do
    for t in $tasks; do
      if [ $v = cur ]; then unset H12ENV_LIB; else export H12ENV_LIB=$PWD/h1v2-isaac_amd/h12env/libh12env_$v.so; fi
      timeout -k 10 240 python -u bench.py --task $t --no-cpu-baseline > $o/bench_${t}_${v}$r.json 2>&1 || { echo "bench $t $v failed"; tail -5 $o/bench_${t}_${v}$r.json; exit 1; }
      python3 -c "import json; d=json.loads(open('$o/bench_${t}_${v}$r.json').read().strip().splitlines()[-1]); print('$t $v', $r, round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step', 'env', round(d['roofline']['kernel_ms_avg']*1e3,2))"
    done
  done
done
