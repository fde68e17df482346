"""GPU parity of the CaT task (row f4, Isaac-Velocity-CaT-Flat-H12_12dof-v0) through the C-ABI against the
oracle: the constraint values of step_kernel, cat_reduce_kernel's running maxima and no_move remap,
cat_prob_kernel's probabilities / reward scaling / dones / episode statistics, the foot-clearance swing state.
Tolerances as in test_gpu_parity.py (>= 99 % of envs at 2e-3 after contact-rich steps: an fp32 contact
decision that flips moves a column maximum, which rescales that column's probabilities in every env)."""
import numpy as np
import pytest
import torch

import oracle as O
from h12env._abi import F as FIELDS
from h12env.cfg import H12CaTEnvCfg
from h12env.env import H12VelocityEnv

pytestmark = pytest.mark.gpu


def field(Fm, k):
    o, c = FIELDS[k]
    return Fm[o:o + c]


def close(a, b, tol=2e-3):
    return np.abs(a - b) <= tol * np.maximum(1, np.abs(b))


def test_cat_steps_match_oracle(gpu):
    n = 512
    cfg = H12CaTEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    ref = O.OracleEnv(env._model, env._ccfg, n)
    ref.F[:] = env._fstate.cpu().numpy()
    ref.I[:] = env._istate.cpu().numpy()
    O.set_dz_count(0)
    O.cat_reset()
    obs, _ = env.reset()
    r = ref.reset()
    np.testing.assert_allclose(obs["policy"].cpu().numpy(), r, rtol=1e-5, atol=2e-5)
    rng = np.random.default_rng(41)
    for t in range(1, 6):
        a = (0.3 * rng.normal(size=(n, 12))).astype(np.float32)
        # modify_constraint_p: both sides use the max_p of counter t - 1
        for name, cid in cfg.constraints.active():
            if name != "contact":
                ref.cfg.cstr_max_p[cid] = 1.0 / (20 + min((t - 1) / 120000, 1.0) * (4 - 20))
        obs, rew, dones, trunc, ext = env.step(torch.from_numpy(a).cuda())
        r_obs, r_rew, r_term, r_trunc, info = ref.step(a, t)
        assert dones.dtype == torch.float32
        d = dones.cpu().numpy()
        assert close(d, info["cstr_prob"], 1e-3).mean() >= 0.99, t
        assert close(rew.cpu().numpy(), r_rew, 1e-3).mean() >= 0.99, t
        assert close(obs["policy"].cpu().numpy(), r_obs).all(axis=1).mean() >= 0.99, t
        g = env._fstate.cpu().numpy()
        for k in ("CSTR_SUM", "CSTR_P", "SWING_H"):
            assert close(field(g, k), field(ref.F, k), 1e-3).all(axis=0).mean() >= 0.99, (t, k)
        assert (d > 0).mean() > 0.05       # constraints are active in the first steps
    keys = list(ext["log"].keys())
    assert "Episode_Constraint_violation/foot_clearance" in keys
    assert "Episode_Constraint_probability/no_move" in keys
    assert abs(env.constraint_manager.get_term_cfg("no_move").max_p - 1 / (20 - 16 * 4 / 120000)) < 1e-9
    env.close()
