"""GPU probe: run-to-run determinism of the env step -- two handles, same seeds and actions, stepped alternately;
prints the first step / envs where rewards, dones or observations differ.  usage: determinism.py TASK N STEPS"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "h1v2-isaac_amd"))
import torch  # noqa: E402

from h12env import H12FlatEnvCfg  # noqa: E402
from h12env.cfg import H12CaTEnvCfg, H12RslEnvCfg  # noqa: E402
from h12env.env import H12VelocityEnv  # noqa: E402

task, n, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
fn = {"flat": H12FlatEnvCfg, "cat": H12CaTEnvCfg, "rsl": H12RslEnvCfg}[task]


def make():
    cfg = fn()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    g = torch.Generator(device="cpu").manual_seed(n)
    env.episode_length_buf = torch.randint(env.max_episode_length - 20, env.max_episode_length, (n,), generator=g,
                                           dtype=torch.int32)
    return env


a, b = make(), make()
gen = torch.Generator(device="cpu").manual_seed(11)
for t in range(steps):
    act = (torch.randn(n, 12, generator=gen) * (0.02 if t % 3 == 0 else 0.4)).cuda()
    oa, ra, ta, ua, _ = a.step(act)
    ob, rb, tb, ub, _ = b.step(act)
    dr = torch.nonzero(ra != rb).flatten()
    do = torch.nonzero((oa["policy"] != ob["policy"]).any(dim=1)).flatten()
    if len(dr) or len(do) or not torch.equal(ta, tb):
        fa, fb = a._fstate, b._fstate
        dfield = torch.nonzero((fa != fb).any(dim=1)).flatten().tolist()
        print(task, "first diff at step", t, "rew envs", dr[:8].tolist(), "obs envs", do[:8].tolist(),
              "state rows differing", dfield[:20], flush=True)
        if len(dr):
            i = dr[:3]
            print("  ra", ra[i].tolist(), "rb", rb[i].tolist(), flush=True)
        break
else:
    print(task, n, steps, "deterministic", flush=True)
