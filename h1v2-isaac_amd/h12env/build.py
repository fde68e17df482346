"""Build libh12env.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m h12env.build            # from h1v2-isaac_amd/
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
SRC_ROOT = PKG.parent
REPO = SRC_ROOT.parent
CSRC = SRC_ROOT / "csrc"
OUT = PKG / "libh12env.so"
ARCH = os.environ.get("H12_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build libh12env.so)")


def sources():
    return [CSRC / "h12env.hip", CSRC / "h12_math.h", CSRC / "h12_model_gen.h", REPO / "include" / "h12env.h"]


def source_sha256() -> str:
    """sha256 over every file the kernels are compiled from (csrc/*.hip, csrc/*.h, include/*.h; path + contents, in
    sorted order): the key profiles/latest_isa.json and the PMC summaries are checked against, so a header-only change
    (e.g. h12_math.h) also marks them stale."""
    import hashlib

    h = hashlib.sha256()
    files = sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.h")) + list((REPO / "include").glob("*.h")))
    for f in files:
        h.update(f.relative_to(REPO).as_posix().encode() + b"\0")
        h.update(f.read_bytes())
    return h.hexdigest()


def needs_build() -> bool:
    if not OUT.exists():
        return True
    t = OUT.stat().st_mtime
    return any(s.stat().st_mtime > t for s in sources())


def build(force: bool = False, verbose: bool = True, extra_flags: list[str] | None = None) -> Path:
    # regenerate the constexpr model header from the committed JSON (pure data)
    subprocess.run([sys.executable, str(REPO / "tools" / "gen_model_header.py")], check=True,
                   stdout=subprocess.DEVNULL)
    if not force and not needs_build():
        return OUT
    # -fno-slp-vectorize: packed-fp32 SLP code needs register pairs and costs ~30 % extra v_mov here.
    # -ffinite-math-only -fno-signed-zeros: the state is finite by construction, so products with
    # the model's zero constants fold away and fminf/fmaxf need no NaN canonicalisation (-21 % VALU
    # in the inner physics step); results of finite operations are unchanged.  Device code only: the
    # host-side config validation keeps its NaN checks.
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fno-slp-vectorize", "-Xarch_device",
           "-ffinite-math-only", "-Xarch_device", "-fno-signed-zeros", "-fPIC", "-shared", "-Wall",
           "-Wno-unused-function", "-o", str(OUT), str(CSRC / "h12env.hip")]
    if extra_flags:
        cmd += extra_flags
    if verbose:
        print("[h12env.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
