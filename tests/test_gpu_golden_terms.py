"""GPU: step_kernel's term code (through the C-ABI parity hook h12env_eval_terms) against the reference's OWN
term functions -- the fixtures tests/test_golden_terms.py pins the oracle with (tools/gen_golden_terms.py):
feet_air_time_positive_biped (velocity/mdp/rewards.py:38-62), action_rate_l2 (utils/mdp/rewards.py:23-30) and the
ten CaT constraint functions of utils/cat/constraints.py (raw values as CaT.add sees them, foot_clearance's swing
state carried over the steps in the workspace).  States are written into the workspace views; fp32 on both sides.
"""
from pathlib import Path

import numpy as np
import pytest
import torch

from h12env import H12FlatEnvCfg
from h12env._abi import CONSTRAINT_TERMS, F, I
from h12env.cfg import H12CaTEnvCfg
from h12env.env import H12VelocityEnv

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"
R_ACTION_RATE, R_FEET_AIR_TIME = 5, 6


def put(env, name, vals):
    o, k = F[name]
    env._fstate[o:o + k] = torch.as_tensor(np.asarray(vals, np.float32).reshape(-1, k).T.copy(), device=env.device)


def make(cfg, n):
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    torch.cuda.synchronize()
    return env


def test_kernel_rewards_match_reference_functions(gpu):
    d = np.load(G / "ref_rewards.npz")
    n = d["cmd"].shape[0]
    env = make(H12FlatEnvCfg(), n)
    env._fstate.zero_()
    put(env, "QUAT", np.tile([1.0, 0, 0, 0], (n, 1)))
    put(env, "POS", np.tile([0.0, 0, 1.0], (n, 1)))
    put(env, "ACT", d["act"])
    put(env, "ACT_PREV", d["act_prev"])
    put(env, "CMD", d["cmd"])
    put(env, "AIR", d["air"])
    put(env, "CONTACT", d["con"])
    z = torch.zeros(n, 12)
    terms, _, _, _ = env.eval_terms(z, z, torch.zeros(n, 5))
    terms = terms.cpu().numpy()
    assert (terms[R_FEET_AIR_TIME] == d["feet_air_time_positive_biped"]).all()
    np.testing.assert_allclose(terms[R_ACTION_RATE], d["action_rate_l2"], rtol=2e-6, atol=1e-6)
    env.close()


def test_kernel_constraints_match_reference_functions(gpu):
    d = np.load(G / "ref_constraints.npz")
    T, n = d["q"].shape[:2]
    cfg = H12CaTEnvCfg()
    cfg.robot.joint_effort_limits_sim = tuple(float(x) for x in d["effort_limits"])
    cfg.robot.joint_vel_limits = tuple(float(x) for x in d["vel_limits"])
    env = make(cfg, n)
    env._fstate.zero_()
    assert [CONSTRAINT_TERMS.index(str(x)) for x in d["term_names"]] == list(range(10))
    for t in range(T):
        put(env, "POS", d["pos"][t])
        put(env, "QUAT", d["quat"][t])
        put(env, "Q", d["q"][t])
        put(env, "QD", d["qd"][t])
        put(env, "CMD", d["cmd"][t])
        put(env, "CONTACT", d["con"][t])
        env._istate[I["EPLEN"][0]] = torch.as_tensor(d["eplen"][t], dtype=torch.int32, device=env.device)
        fn = np.linalg.norm(d["forces"][t], axis=-1).max(axis=1)  # max over the history of |F|, per body
        fmax = np.concatenate([fn[:, 3:5], fn[:, 0:2], fn[:, 2:3]], 1)
        _, term, _, cs = env.eval_terms(torch.as_tensor(d["tau"][t]), torch.zeros(n, 12), torch.as_tensor(fmax))
        cs = cs.cpu().numpy()
        raw = d["raw"][t]                                   # (n, 56) as CaT.add saw them (no_move remapped)
        still = (np.abs(d["cmd"][t]) < 0.2).all(axis=1)
        assert (cs[57] == d["eplen"][t]).all() and (cs[56].astype(bool) == still).all()
        atol = np.full(56, 4e-6)
        atol[25:37], atol[37:39] = 6e-5, 6e-4               # |x| - limit at fp32 (torques ~1e2, forces ~1e3)
        nm = slice(39, 51)
        own = np.ones(56, bool)
        own[nm] = False
        err = np.abs(cs[:56].T - raw)[:, own]
        assert (err <= (atol + 2e-6 * np.abs(raw))[:, own]).all(), (t, np.argwhere(err > atol[own]))
        # no_move: the reference hands env i the row of the (i mod m)-th still env
        ids = np.nonzero(still)[0]
        if len(ids):
            src = ids[np.arange(n) % len(ids)]
            np.testing.assert_allclose(cs[nm][:, src].T, raw[:, nm], rtol=2e-6, atol=4e-6)
        assert (cs[0].astype(bool) == (raw[:, 0] > 0)).all() and (term.cpu().numpy() == (raw[:, 0] > 0)).all()
        # the hook leaves the workspace's swing state alone and returns the updated one: carry it like a step
        sw_ws = env._fstate[F["SWING_H"][0]:F["SWING_H"][0] + 2].clone()
        _, _, _, cs2 = env.eval_terms(torch.as_tensor(d["tau"][t]), torch.zeros(n, 12), torch.as_tensor(fmax))
        assert torch.equal(env._fstate[F["SWING_H"][0]:F["SWING_H"][0] + 2], sw_ws)   # read-only hook
        assert np.array_equal(cs2.cpu().numpy(), cs)                                   # so a repeat is identical
        env._fstate[F["SWING_H"][0]:F["SWING_H"][0] + 2] = torch.as_tensor(cs[58:60], device=env.device)
    sw = env._fstate[F["SWING_H"][0]:F["SWING_H"][0] + 2].T.cpu().numpy()
    np.testing.assert_allclose(sw, d["swing_max_height_final"], rtol=2e-6, atol=2e-6)
    env.close()
