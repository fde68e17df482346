"""GPU probe: is each CaT path deterministic run to run?  Two handles of the same path, same seeds and actions,
stepped alternately; reports the first step where their rewards / dones / observations differ."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "h1v2-isaac_amd"))
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "tests"))
import torch  # noqa: E402
from test_gpu_cat_inline import _make  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
for inline in (True, False):
    a, b = _make(n, inline), _make(n, inline)
    gen = torch.Generator(device="cpu").manual_seed(11)
    first = None
    for t in range(steps):
        act = (torch.randn(n, 12, generator=gen) * (0.02 if t % 3 == 0 else 0.4)).cuda()
        oa, ra, ta, ua, _ = a.step(act)
        ob, rb, tb, ub, _ = b.step(act)
        same = torch.equal(ra, rb) and torch.equal(ta, tb) and torch.equal(oa["policy"], ob["policy"])
        if not same and first is None:
            first = t
            d = torch.nonzero(ra != rb).flatten()
            print("inline" if inline else "two-kernel", "first diff at step", t, "rew envs", d[:10].tolist(),
                  "blocks", (d // 32).unique().tolist()[:10], "dones differ", int((ta != tb).sum()), flush=True)
    print("inline" if inline else "two-kernel", "deterministic" if first is None else "NOT deterministic", flush=True)
    for e in (a, b):
        try:
            e.close()
        except Exception as ex:  # noqa: BLE001
            print("close:", ex)
