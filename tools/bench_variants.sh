#!/bin/bash
# Task-variant and PPO bench lines for DESIGN.md §5 (GPU box, repo root): bash tools/bench_variants.sh <tag>
set -o pipefail
TAG=${1:-variants}
mkdir -p gpurun_out
OUT=gpurun_out/variants_$TAG.log
: > $OUT
for t in rsl cat rough c5; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --task $t --steps 500 > gpurun_out/b_$t.log 2>&1 || { echo "bench $t failed"; tail -5 gpurun_out/b_$t.log; exit 1; }
  echo "$t $(tail -1 gpurun_out/b_$t.log)" >> $OUT
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-self-collision --steps 500 > gpurun_out/b_noself.log 2>&1 && echo "noself $(tail -1 gpurun_out/b_noself.log)" >> $OUT
timeout -k 10 400 python -u bench.py --no-cpu-baseline --mode train > gpurun_out/b_train.log 2>&1 && echo "train $(tail -1 gpurun_out/b_train.log)" >> $OUT
timeout -k 10 400 python -u bench.py --no-cpu-baseline --mode train --precision bf16 > gpurun_out/b_train_bf16.log 2>&1 && echo "train_bf16 $(tail -1 gpurun_out/b_train_bf16.log)" >> $OUT
python3 - "$OUT" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    tag, js = line.split(" ", 1)
    d = json.loads(js)
    r = d.get("roofline", {})
    print(tag, round(d["value"] / 1e6, 2), "M", round(d["ms_per_step"] * 1e3, 1), "us/step", r.get("kernel_ms_avg"), (r.get("secondary") or {}).get("kernel_ms_avg"))
PY
