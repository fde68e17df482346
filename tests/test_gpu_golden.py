"""GPU: the HIP kernels against the reference-generated golden vectors (tests/golden, see
tools/gen_golden.py) through the C-ABI (h12env_observe, h12env_reset)."""
from pathlib import Path

import numpy as np
import pytest
import torch

from h12env import H12FlatEnvCfg
from h12env._abi import F
from h12env.env import H12VelocityEnv

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def env_no_noise(n):
    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    cfg.observations.policy.enable_corruption = False
    env = H12VelocityEnv(cfg)
    env.reset()
    return env


def put(env, name, vals):
    o, k = F[name]
    env._fstate[o:o + k] = torch.as_tensor(np.asarray(vals, np.float32).T.reshape(k, -1), device="cuda:0")


def test_kernel_observation_matches_deploy_handler(gpu):
    z = np.load(GOLD / "deploy_obs.npz")
    env = env_no_noise(1)
    for t in range(z["obs"].shape[0]):
        put(env, "QUAT", z["quat"][t][None])
        put(env, "WANG", z["wang"][t][None])
        put(env, "CMD", z["cmd"][t][None])
        put(env, "Q", z["q"][t][None])
        put(env, "QD", z["qd"][t][None])
        put(env, "ACT", z["act"][t][None])
        obs = env.observe(torch.tensor([t == 0], dtype=torch.uint8))["policy"]
        np.testing.assert_allclose(obs.cpu().numpy()[0], z["obs"][t], rtol=2e-6, atol=2e-6)
    env.close()


def test_kernel_history_matches_circular_buffer(gpu):
    z = np.load(GOLD / "circular_buffer.npz")
    q0 = None
    for d, name, off in ((3, "WANG", 0), (12, "Q", 90)):
        frames, resets, hist = z[f"frames_d{d}"], z[f"resets_d{d}"], z[f"history_d{d}"]
        T, n = resets.shape
        env = env_no_noise(n)
        q0 = np.array(env._model.q_default, np.float32)
        for t in range(T):
            vals = frames[t] + (q0 if name == "Q" else 0)
            put(env, name, vals)
            fill = torch.as_tensor((resets[t] | (t == 0)).astype(np.uint8))
            obs = env.observe(fill)["policy"].cpu().numpy()
            got = obs[:, off:off + 10 * d].reshape(n, 10, d)
            if name == "Q":
                np.testing.assert_allclose(got, hist[t], rtol=0, atol=3e-7)  # (q0 + x) - q0 in fp32
            else:
                np.testing.assert_array_equal(got, hist[t])
        env.close()
