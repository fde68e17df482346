"""Fold tools/profile.sh's rocprofv3 CSVs into profiles/<tag>_pmc.json and profiles/latest_pmc.json.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half the bytes of wide
reads: /opt/skills/guides/MI355X_MICROARCH.md, HBM section).  Only the timed-loop dispatches of the
two step kernels are used (the profile-only bench run launches nothing else of ours at that rate).
"""
from __future__ import annotations

import csv
import glob
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))
from h12env.build import source_sha256  # noqa: E402
KERNELS = ("step_kernel", "obs_assemble_kernel")


def short(name: str) -> str | None:
    for k in KERNELS:
        if k in name:
            return k
    return None


def counters(d: Path):
    """{kernel: {counter: [per-dispatch values]}} from *counter_collection.csv"""
    out = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if not k:
                    continue
                out[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                meta[k] = {x: row.get(x) for x in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size",
                                                   "LDS_Block_Size", "Workgroup_Size", "Grid_Size") if x in row}
    return out, meta


def mean(v):
    return sum(v) / len(v) if v else None


def main():
    src, tag = Path(sys.argv[1]), sys.argv[2]
    res = {"tag": tag, "source_sha256": source_sha256(),
           "command": "bash tools/profile.sh (rocprofv3 --pmc <counters> --kernel-trace -f csv -- python3 bench.py "
                      "--steps 100 --warmup 20 --no-cpu-baseline --profile-only)",
           "kernels": {}}
    # the device ISA the counters belong to (tools/kernel_isa.py --json, when made from this same source): a later
    # source edit that leaves the ISA unchanged (comments, profile-only macros) keeps the counters valid
    isa = ROOT / "profiles" / "latest_isa.json"
    if isa.exists():
        d = json.loads(isa.read_text())
        if d.get("source_sha256") == res["source_sha256"]:
            res["isa_sha256"] = d.get("isa_sha256")
    fetch, meta = counters(src / "fetch")
    write, _ = counters(src / "write")
    sq, _ = counters(src / "sq")
    for k in KERNELS:
        # counters are summed over the dispatch's XCDs / instances per row: aggregate per dispatch count
        f = fetch.get(k, {}).get("FETCH_SIZE", [])
        w = write.get(k, {}).get("WRITE_SIZE", [])
        n_f = len(f) or 1
        fkb = mean(f)
        wkb = mean(w)
        ent = {"dispatches": len(f), "FETCH_SIZE_KB_raw": fkb, "WRITE_SIZE_KB": wkb, **meta.get(k, {})}
        if fkb is not None and wkb is not None:
            ent["hbm_read_bytes_per_launch"] = 2.0 * fkb * 1024.0
            ent["hbm_write_bytes_per_launch"] = wkb * 1024.0
            ent["hbm_bytes_per_launch"] = ent["hbm_read_bytes_per_launch"] + ent["hbm_write_bytes_per_launch"]
        ent["SQ"] = {c: mean(v) for c, v in sq.get(k, {}).items()}
        res["kernels"][k] = ent
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)
    txt = json.dumps(res, indent=1)
    (prof / f"{tag}_pmc.json").write_text(txt)
    (prof / "latest_pmc.json").write_text(txt)
    stats = glob.glob(str(src / "stats" / "**" / "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], prof / f"{tag}_kernel_stats.csv")
    print(txt)


if __name__ == "__main__":
    main()
