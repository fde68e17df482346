#!/bin/bash
# GPU box: one bench line per task / mode of the in-tree library, summarised into gpurun_out/<tag>_task_lines.txt
# (the DESIGN / README task figures).  Usage: bash tools/task_lines.sh <tag>
set -o pipefail
tag=${1:-tasks}
o=gpurun_out/$tag
mkdir -p $o
sum=gpurun_out/${tag}_task_lines.txt
: > $sum
line() {  # name, json file
  python3 - "$1" "$2" >> $sum <<'PY'
import json, sys
name, f = sys.argv[1], sys.argv[2]
d = json.loads(open(f).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
if "learning_s_per_iter" in d:
    print(name, round(d["value"] / 1e6, 3), "M", "learn", round(d["learning_s_per_iter"] * 1e3, 1), "ms collect",
          round(d["collection_s_per_iter"] * 1e3, 2), "ms per iteration")
else:
    sec = r.get("secondary") or {}
    print(name, round(d["value"] / 1e6, 2), "M", round(d["ms_per_step"] * 1e3, 2), "us/step env",
          round(r.get("kernel_ms_avg", 0) * 1e3, 2), "second", round(sec.get("kernel_ms_avg", 0) * 1e3, 2))
PY
}
for t in rsl cat rough c5; do
  timeout -k 10 240 python3 -u bench.py --task $t --no-cpu-baseline > $o/bench_$t.json 2> $o/bench_$t.err || { echo "bench $t failed"; exit 1; }
  line $t $o/bench_$t.json
done
timeout -k 10 240 python3 -u bench.py --rollout on --no-cpu-baseline > $o/bench_rollout.json 2> $o/bench_rollout.err || { echo "rollout failed"; exit 1; }
line "rollout on" $o/bench_rollout.json
timeout -k 10 240 python3 -u bench.py --steps 20 --warmup 5 > $o/bench_drv.json 2> $o/bench_drv.err || { echo "driver cmd failed"; exit 1; }
line "driver cmd" $o/bench_drv.json
timeout -k 10 400 python3 -u bench.py --mode train --no-cpu-baseline > $o/bench_train.json 2> $o/bench_train.err || { echo "train failed"; exit 1; }
line train $o/bench_train.json
timeout -k 10 400 python3 -u bench.py --mode train --tunableop --no-cpu-baseline > $o/bench_train_tunable.json 2> $o/bench_train_tunable.err || { echo "train tunableop failed"; exit 1; }
line "train tunableop" $o/bench_train_tunable.json
cat $sum
