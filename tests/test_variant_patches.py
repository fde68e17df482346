"""CPU: every experiment patch in tools/variant.py (the measured-and-not-kept variants and the slack probes DESIGN.md
section 5 cites) applies to the kernel source it was written for -- the round-4 patches to commit R4_BASE's source,
the others to the working tree -- with its expected number of matches, and changes that source, so the recorded A/Bs
stay reproducible."""
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import variant  # noqa: E402


def _have_rev(rev):
    if rev is None:
        return True
    r = subprocess.run(["git", "cat-file", "-e", f"{rev}^{{commit}}"], cwd=ROOT, capture_output=True)
    return r.returncode == 0


@pytest.mark.parametrize("tag", sorted(variant.ALL))
def test_patch_applies(tag):
    rev, patches = variant.ALL[tag]
    if not _have_rev(rev):
        pytest.skip(f"git history with {rev} not available")
    src = variant.source_at(rev, variant.SOURCES[0])
    for old, new, *cnt in patches:
        assert src.count(old) == (cnt[0] if cnt else 1), (tag, old[:60])
        assert old != new
        nxt = src.replace(old, new)
        assert nxt != src, (tag, old[:60])
        src = nxt
    orig, out = variant.patched(tag)
    assert out != orig and out == src
