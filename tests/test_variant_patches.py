"""CPU: every experiment patch in tools/variant.py (the measured-and-not-kept variants and the slack probes DESIGN.md
section 5 cites) still applies to the product kernel source with its expected number of matches, so the recorded
A/Bs stay reproducible."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import variant  # noqa: E402


@pytest.mark.parametrize("tag", sorted(variant.PATCHES))
def test_patch_applies(tag):
    src = (ROOT / "h1v2-isaac_amd" / "csrc" / "h12env.hip").read_text()
    for old, new, *cnt in variant.PATCHES[tag]:
        assert src.count(old) == (cnt[0] if cnt else 1), (tag, old[:60])
        src = src.replace(old, new)
