# round 5: A/B of the in-tree library against variants, then FETCH / WRITE PMC passes of each (H12ENV_LIB)
set -o pipefail
tag=$1; shift
bash tools/ab_run.sh ${tag}_ab 3 - "$@" || exit 1
export TMPDIR=/tmp
B="python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --profile-only"
for v in new "$@"; do
  unset H12ENV_LIB
  [ "$v" != new ] && export H12ENV_LIB=$PWD/tools/_variants/lib_$v.so
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 200 rocprofv3 --pmc $c --kernel-trace -f csv -d gpurun_out/${tag}_pmc_$v/$c -o run -- $B > gpurun_out/${tag}_pmc_${v}_$c.log 2>&1 || { echo "pmc $v $c failed"; exit 1; }
  done
done
unset H12ENV_LIB
python3 - "$tag" "$@" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
for v in ["new"] + sys.argv[2:]:
    out = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = []
        for f in glob.glob(f"gpurun_out/{tag}_pmc_{v}/{c}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                if "step_kernel" in row["Kernel_Name"] and row["Counter_Name"] == c:
                    vals.append(float(row["Counter_Value"]))
        out[c] = sum(vals) / max(1, len(vals))
    print(v, "read MB (2x FETCH)", round(2 * out["FETCH_SIZE"] * 1024 / 1e6, 3), "write MB", round(out["WRITE_SIZE"] * 1024 / 1e6, 3))
PY
