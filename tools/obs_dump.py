"""GPU: observations of a few seeded steps of one task (tests pick the library with H12ENV_LIB) -> a .pt file, for
bit-for-bit A/B comparisons of kernel variants.  Usage: python tools/obs_dump.py <task rough|c5|flat> <n> <out.pt>"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "h1v2-isaac_amd"))
from h12env import H12FlatEnvCfg  # noqa: E402
from h12env.cfg import H12RoughEnvCfg, c5_cfg  # noqa: E402
from h12env.env import H12VelocityEnv  # noqa: E402

task, n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
cfg = H12FlatEnvCfg() if task == "flat" else H12RoughEnvCfg()
if task == "c5":
    cfg = c5_cfg()
cfg.scene.num_envs = n
cfg.sim.device = "cuda:0"
env = H12VelocityEnv(cfg)
obs, _ = env.reset()
res = [obs["policy"].clone()]
g = torch.Generator(device="cpu").manual_seed(5)
for _ in range(6):
    o, r, te, tr, _ = env.step(torch.randn(n, 12, generator=g).cuda())
    res += [o["policy"].clone(), r.clone()]
torch.save([x.cpu() for x in res], out)
print("saved", out, len(res))
