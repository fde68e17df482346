#!/usr/bin/env python3
"""GPU diagnostic: kernel self-contact wrenches (h12env_eval_self_contacts) against the oracle's on given physics
states (tools/_selfdiag.npz: S (k, 37) fp64 states, tags), each state rounded to fp32 first so that only the
kernel's arithmetic differs.  Prints the states whose wrench error exceeds 1e-4 of the largest wrench entry."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "h1v2-isaac_amd"), str(ROOT / "oracle"), str(ROOT / "tests" / "helpers")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from h12env import H12FlatEnvCfg  # noqa: E402
from h12env.env import H12VelocityEnv  # noqa: E402

d = np.load(sys.argv[1] if len(sys.argv) > 1 else ROOT / "tools" / "_selfdiag.npz")
S, tags = d["S"], d["tags"]
n = S.shape[0]
cfg = H12FlatEnvCfg()
cfg.scene.num_envs = n
cfg.sim.device = "cuda:0"
env = H12VelocityEnv(cfg)
env.reset()
Fm = env._fstate.cpu().numpy().copy()
Fm[0:37] = S.T.astype(np.float32)
env._fstate.copy_(torch.from_numpy(Fm))
g = env.eval_self_contacts().cpu().numpy().astype(np.float64)
bodies = [(0, 0, 4), (0, 1, 6), (1, 0, 10), (1, 1, 12)]
np.set_printoptions(precision=5, suppress=True, linewidth=220)
rows = []
for i in range(n):
    s = Fm[0:37, i].astype(np.float64)
    f, _ = O.self_contacts(env._model, env._ccfg, s)
    scale = max(1.0, np.abs(f).max())
    err = max(np.abs(g[i, leg, b] - f[body]).max() / scale for leg, b, body in bodies)
    rows.append((err, i))
    if err > 1e-4:
        print(f"{tags[i]} err {err:.2e} scale {scale:.1f}")
        for leg, b, body in bodies:
            if np.abs(f[body]).max() > 0 or np.abs(g[i, leg, b]).max() > 0:
                print(f"   body {body} gpu {g[i, leg, b]}\n           orc {f[body]}")
e = np.array([r[0] for r in rows])
print("quantiles 0.5/0.9/0.99/max", np.quantile(e, [0.5, 0.9, 0.99, 1.0]), "states", n,
      "with contact", int(sum(1 for i in range(n) if True)))
env.close()
