#!/usr/bin/env python3
"""Static ISA report of libh12env's kernels (gfx950): register allocation from the code-object metadata and
instruction counts from the compiler's own assembly.

    python tools/kernel_isa.py [kernel-name-substring ...] [--json profiles/latest_isa.json]

Builds csrc/h12env.hip with -save-temps into a temp dir (same flags as h12env.build), then for each kernel
prints .vgpr_count / .agpr_count / .sgpr_count / scratch, the instruction mix (VALU, v_accvgpr moves, SALU,
vector / scalar memory, s_waitcnt) and every loop body (backward branch) with its VALU count.

Register accounting on gfx950: one wave has up to 512 registers per lane, arch VGPRs first then AGPRs (unified
file; .agpr_count > 0 only when the allocator spills into AGPRs, each use costing a v_accvgpr_read/write).
rocprofv3's "VGPR_Count" / "Accum_VGPR_Count" columns report the dispatch's granule-rounded arch VGPR /
AGPR fields, which is why they can differ from the metadata here.
"""
from __future__ import annotations

import re
import subprocess
import sys
import tempfile
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))


def build_asm(tmp: Path) -> Path:
    from h12env.build import ARCH, CSRC, hipcc

    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fno-slp-vectorize", "-Xarch_device",
           "-ffinite-math-only", "-Xarch_device", "-fno-signed-zeros", "-fPIC", "-shared", "-save-temps",
           "-Wno-unused-function", "-o", str(tmp / "lib.so"), str(CSRC / "h12env.hip")]
    subprocess.run(cmd, check=True, cwd=tmp, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    s = sorted(tmp.glob(f"*{ARCH}*.s"))
    if not s:
        raise RuntimeError("no device assembly produced")
    return s[0]


def metadata(text: str) -> dict:
    import yaml

    y = text.split("\n\t.amdgpu_metadata", 1)[1].split("\t.end_amdgpu_metadata", 1)[0]
    out = {}
    for k in yaml.safe_load(y)["amdhsa.kernels"]:
        out[k[".name"]] = {key[1:]: v for key, v in k.items() if isinstance(v, int)}
    return out


def report(text: str, name: str) -> dict:
    lines = text.splitlines()
    i0 = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    i1 = next(i for i in range(i0, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[i0:i1]
    ins = [l.strip().split()[0] for l in body if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    c = Counter(ins)
    r = {"total": len(ins), "valu": sum(v for k, v in c.items() if k.startswith("v_")),
         "accvgpr": sum(v for k, v in c.items() if k.startswith("v_accvgpr")),
         "salu": sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith(("s_waitcnt", "s_load",
                                                                                          "s_buffer"))),
         "vmem": sum(v for k, v in c.items() if k.startswith(("buffer_", "global_", "flat_"))),
         "smem": sum(v for k, v in c.items() if k.startswith(("s_load", "s_buffer_load"))),
         "waitcnt": c["s_waitcnt"], "loops": []}
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB[\d_]+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB[\d_]+)|s_branch\s+(\.LBB[\d_]+)", l)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i:
                seg = [x.strip().split()[0] for x in body[labels[tgt]:i]
                       if x.startswith("\t") and x.strip() and not x.strip().startswith((".", ";"))]
                cc = Counter(seg)
                r["loops"].append((tgt, len(seg), sum(v for k, v in cc.items() if k.startswith("v_")),
                                   sum(v for k, v in cc.items() if k.startswith("v_accvgpr")), cc["s_waitcnt"]))
    return r


def isa_sha256(text: str) -> str:
    """sha256 of the device assembly with comments and the per-source compile-unit id (__hip_cuid_*) removed: equal
    for two sources that compile to the same machine code (e.g. after a comment-only or dead-macro edit)."""
    import hashlib
    import re

    lines = []
    for ln in text.splitlines():
        if ln.lstrip().startswith(";") or ln.startswith("\t.file") or ".ident" in ln:
            continue
        lines.append(re.sub(r"__hip_cuid_[0-9a-f]+", "__hip_cuid", ln.split(";")[0].rstrip()))
    return hashlib.sha256("\n".join(lines).encode()).hexdigest()


def physics_wave_json(text: str, meta: dict, out: Path) -> None:
    """profiles/latest_isa.json for bench.py's issue roofline: the Flat step_kernel's register allocation and the
    VALU count of its physics wave's physics-step loop, keyed by the kernel source's sha256 like latest_pmc.json.
    The physics wave is the one whose registers overflow into AGPRs, so its loop is the one with the most
    v_accvgpr moves (largest VALU count among ties); the helper / self-contact loops use none and, with the fused
    observation stores, the helper loop has more VALU than the physics loop."""
    import json

    from h12env.build import source_sha256

    name = next(k for k in meta if "step_kernelILi0E" in k)
    g, r = meta[name], report(text, name)
    top = max(r["loops"], key=lambda x: (x[3], x[2]))
    res = {"source_sha256": source_sha256(),
           "kernel": name,
           "registers": {"vgpr_count_total": g.get("vgpr_count"), "agpr_count": g.get("agpr_count"),
                         "arch_vgpr": (g.get("vgpr_count") or 0) - (g.get("agpr_count") or 0),
                         "sgpr_count": g.get("sgpr_count"), "scratch_bytes": g.get("private_segment_fixed_size"),
                         "note": "gfx950 unified file: .vgpr_count is arch + acc registers; rocprofv3's VGPR_Count "
                                 "column decodes the descriptor's granulated field with a granule of 4 instead of 8 "
                                 "(half the allocated count)"},
           "physics_step_loop": {"label": top[0], "instructions": top[1], "valu": top[2], "v_accvgpr": top[3]},
           "valu_total_static": r["valu"], "isa_sha256": isa_sha256(text)}
    out.write_text(json.dumps(res, indent=1) + "\n")
    print("wrote", out)


def main():
    args = sys.argv[1:]
    js = None
    if "--json" in args:
        i = args.index("--json")
        js = Path(args[i + 1])
        del args[i:i + 2]
    subs = args or ["step_kernelILi0E", "obs_assemble_kernelILi10E"]
    with tempfile.TemporaryDirectory() as td:
        text = build_asm(Path(td)).read_text()
    meta = metadata(text)
    print("isa_sha256", isa_sha256(text))
    if js is not None:
        physics_wave_json(text, meta, js)
    for name, g in sorted(meta.items()):
        if not any(s in name for s in subs):
            continue
        r = report(text, name)
        print(f"{name}: vgpr {g.get('vgpr_count')} agpr {g.get('agpr_count')} sgpr {g.get('sgpr_count')} "
              f"scratch {g.get('private_segment_fixed_size')} B (spills vgpr {g.get('vgpr_spill_count', 0)} "
              f"sgpr {g.get('sgpr_spill_count', 0)})")
        print(f"  instructions {r['total']}: VALU {r['valu']} (v_accvgpr {r['accvgpr']}), SALU {r['salu']}, "
              f"VMEM {r['vmem']}, SMEM {r['smem']}, s_waitcnt {r['waitcnt']}")
        for tgt, n, v, a, w in r["loops"]:
            print(f"  loop {tgt}: {n} instructions, VALU {v}, v_accvgpr {a}, s_waitcnt {w}")


if __name__ == "__main__":
    main()
