#!/bin/bash
# Parameterised A/B on one GPU box (replaces round 4's one-off tools/probe/r4*.sh recipes; they are in git history at
# commit 787ede1).  Optionally a set of GPU test files first (on the in-tree library), then the default bench line
# alternating between the in-tree library ("new") and each named variant library, RUNS rounds.
#
#   bash tools/ab_run.sh <tag> <runs> "<test files or ->" [variant ...]
#
# A variant name v loads tools/_variants/lib_v.so (tools/variant.py) or, if that does not exist,
# h1v2-isaac_amd/h12env/libh12env_v.so (tools/build_variant.sh).  Results: gpurun_out/<tag>_<v><run>.json.
set -o pipefail
tag=$1; runs=$2; tests=$3; shift 3
mkdir -p gpurun_out
if [ -n "$tests" ] && [ "$tests" != "-" ]; then
  timeout -k 10 500 python3 -u -m pytest $tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${tag}_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.txt; exit 1; }
  tail -2 gpurun_out/${tag}_tests.txt
fi
for r in $(seq 1 "$runs"); do
  for v in new "$@"; do
    unset H12ENV_LIB
    if [ "$v" != new ]; then
      lib=$PWD/tools/_variants/lib_$v.so
      [ -f "$lib" ] || lib=$PWD/h1v2-isaac_amd/h12env/libh12env_$v.so
      export H12ENV_LIB=$lib
    fi
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 1000 > gpurun_out/${tag}_$v$r.json 2>/dev/null \
      || { echo "bench $v failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_$v$r.json').read().strip().splitlines()[-1]); print('$v run $r', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us/step step_kernel', round(d['roofline']['kernel_ms_avg']*1e3,2))"
  done
done
unset H12ENV_LIB
