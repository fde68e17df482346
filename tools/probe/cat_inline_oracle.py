"""GPU probe: both CaT paths (inline / two-kernel) against the oracle, per constraint term, with still envs."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from h12env._abi import F as FIELDS  # noqa: E402
from h12env.cfg import H12CaTEnvCfg  # noqa: E402
from h12env.env import H12VelocityEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
for inline in (True, False):
    os.environ["H12_CAT_INLINE"] = "1" if inline else "0"
    cfg = H12CaTEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    ref = O.OracleEnv(env._model, env._ccfg, n)
    ref.F[:] = env._fstate.cpu().numpy()
    ref.I[:] = env._istate.cpu().numpy()
    O.set_dz_count(0)
    O.cat_reset()
    env.reset()
    ref.reset()
    rng = np.random.default_rng(41)
    for t in range(1, 5):
        a = ((0.02 if t % 3 == 1 else 0.3) * rng.normal(size=(n, 12))).astype(np.float32)
        for name, cid in cfg.constraints.active():
            if name != "contact":
                ref.cfg.cstr_max_p[cid] = 1.0 / (20 + min((t - 1) / 120000, 1.0) * (4 - 20))
        env.step(torch.from_numpy(a).cuda())
        ref.step(a, t)
        o, c = FIELDS["CSTR_SUM"]
        g = env._fstate.cpu().numpy()[o:o + c]
        r = ref.F[o:o + c]
        bad = (np.abs(g - r) > 1e-3 * np.maximum(1, np.abs(r))).sum(axis=1)
        print("inline" if inline else "two-kernel", "t", t, "CSTR_SUM envs off per term", bad.tolist(), flush=True)
    env.close()
