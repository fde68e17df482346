set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace -f csv -d gpurun_out/calib/$c -o run -- ./tools/probe/fetch_calib > gpurun_out/calib/$c.log 2>&1 || { echo "$c failed"; tail -5 gpurun_out/calib/$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    d = defaultdict(list)
    for f in glob.glob(f"gpurun_out/calib/{c}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == c:
                d[row["Kernel_Name"].split("(")[0]].append(float(row["Counter_Value"]))
    for k, v in sorted(d.items()):
        print(c, k, "KB", [round(x) for x in v], "factor vs 65536 KB", round(sum(v) / len(v) / 65536, 3))
PY
