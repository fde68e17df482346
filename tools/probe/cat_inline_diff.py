"""GPU probe: where cat_prob_inline and the two-kernel CaT path differ (first steps, 4096 envs)."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "h1v2-isaac_amd"))
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "tests"))
import torch  # noqa: E402
from test_gpu_cat_inline import _make  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
a, b = _make(n, True), _make(n, False)
print("inline", a.cat_inline, b.cat_inline)
gen = torch.Generator(device="cpu").manual_seed(11)
for t in range(3):
    act = (torch.randn(n, 12, generator=gen) * (0.02 if t % 3 == 0 else 0.4)).cuda()
    oa, ra, ta, ua, _ = a.step(act)
    ob, rb, tb, ub, _ = b.step(act)
    dr = (ra - rb).abs()
    dt = (ta - tb).abs()
    bad = torch.nonzero(dr > 0).flatten()
    print(f"t={t} obs_eq={torch.equal(oa['policy'], ob['policy'])} rew ndiff={int((dr > 0).sum())} max={dr.max().item():.3e}"
          f" prob ndiff={int((dt > 0).sum())} max={dt.max().item():.3e} first={bad[:12].tolist()}")
    from h12env._abi import F as FIELDS
    for key in ("CSTR_SUM", "CSTR_P"):
        o, c = FIELDS[key]
        da = (a._fstate[o:o + c] != b._fstate[o:o + c])
        print("  ", key, "per term ndiff", da.sum(dim=1).tolist())
    if len(bad):
        i = bad[:4]
        print("  ra", ra[i].tolist(), "rb", rb[i].tolist())
        print("  ta", ta[i].tolist(), "tb", tb[i].tolist())
        print("  rel", ((ra[i] / rb[i]) - 1).tolist())
for e in (a, b):
    try:
        e.close()
    except Exception as ex:  # noqa: BLE001
        print("close:", ex)
