"""GPU probe: one env's base and joint state magnitudes over the steps of the determinism workload."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "h1v2-isaac_amd"))
import torch  # noqa: E402

from h12env._abi import F  # noqa: E402
from h12env.cfg import H12RslEnvCfg  # noqa: E402
from h12env.env import H12VelocityEnv  # noqa: E402

n, e, t0, t1 = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
cfg = H12RslEnvCfg()
cfg.scene.num_envs = n
cfg.sim.device = "cuda:0"
env = H12VelocityEnv(cfg)
env.reset()
g = torch.Generator(device="cpu").manual_seed(n)
env.episode_length_buf = torch.randint(env.max_episode_length - 20, env.max_episode_length, (n,), generator=g,
                                       dtype=torch.int32)
gen = torch.Generator(device="cpu").manual_seed(11)
for t in range(t1):
    act = (torch.randn(n, 12, generator=gen) * (0.02 if t % 3 == 0 else 0.4)).cuda()
    o, r, d, u, _ = env.step(act)
    if t >= t0:
        f = env._fstate[:, e].cpu()
        def mx(k):
            a, c = F[k]
            return float(f[a:a + c].abs().max())
        print(t, "rew", float(r[e]), "pos", [round(float(x), 3) for x in f[F["POS"][0]:F["POS"][0] + 3]],
              "|v|", round(mx("VLIN"), 2), "|w|", round(mx("WANG"), 2), "|qd|", round(mx("QD"), 1), "term", int(d[e] > 0),
              int(u[e]), flush=True)
