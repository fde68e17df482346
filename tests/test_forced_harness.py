"""CPU tests of the teacher-forced parity harness itself (tests/helpers/forced.py), with the oracle standing in
for the GPU: a stand-in whose only difference is an fp32-scale perturbation of the state must pass (every
off-tolerance env reproduced by the oracle under perturbation), and planted bugs -- a wrong reward term on a
few envs, a wrong joint velocity on every 8th env at one step -- must be reported as unexplained (an error in an
ill-conditioned env-step is legitimately indistinguishable from amplified rounding; the well-conditioned ones are
caught)."""
import numpy as np
import pytest
import torch

import oracle as O
from forced import ForcedParity, perturbed
from h12env import H12FlatEnvCfg
from h12env._abi import F as FIELDS
from h12env.model import build_model


class OracleStandIn:
    """The surface ForcedParity drives (H12VelocityEnv's), backed by the CPU oracle."""

    def __init__(self, n, bug=None, seed=0):
        cfg = H12FlatEnvCfg()
        cfg.scene.num_envs = n
        self._model, self._ccfg = build_model(), cfg.to_c()
        self.num_envs, self.env_offset, self.device = n, 0, torch.device("cpu")
        self.core = O.OracleEnv(self._model, self._ccfg, n)
        self.core.reset()
        self._fstate = torch.from_numpy(self.core.F)
        self._istate = torch.from_numpy(self.core.I)
        self._obs = [torch.from_numpy(self.core.obs)]
        self._k = 0
        self.common_step_counter = 0
        self.bug = bug
        self.rng = np.random.default_rng(seed)

    def step(self, a):
        self.common_step_counter += 1
        self.core.F[:] = perturbed(self.rng, self.core.F, 1e-7)  # fp32-scale "rounding" of the stand-in
        o0, c0 = FIELDS["EPSUM"]
        eps0 = self.core.F[o0:o0 + c0].copy()
        obs, rew, term, trunc, info = self.core.step(a.numpy(), self.common_step_counter)
        if self.bug == "term":   # feet_slide contribution 1 % too large on every 7th env
            m = np.zeros(self.num_envs, bool)
            m[::7] = True
            m &= ~(term | trunc)
            d = self.core.F[o0 + 10] - eps0[10]
            self.core.F[o0 + 10, m] += 0.01 * d[m] - 1e-4
            rew[m] += 0.01 * d[m] - 1e-4
        if self.bug == "qd" and self.common_step_counter == 5:  # every 8th env's knee velocity off by 1 %
            o, _ = FIELDS["QD"]
            self.core.F[o + 3, ::8] *= 1.01
        self._fstate = torch.from_numpy(self.core.F)
        self._istate = torch.from_numpy(self.core.I)
        self._obs = [torch.from_numpy(obs)]
        return {"policy": self._obs[0]}, torch.from_numpy(rew), torch.from_numpy(term), torch.from_numpy(trunc), {}


def run(bug, n=64, steps=25):
    env = OracleStandIn(n, bug)
    fp = ForcedParity(env, seed=1)
    rng = np.random.default_rng(2)
    for _ in range(steps):
        fp.step(rng.normal(size=(n, 12)).astype(np.float32))
    return fp


def test_fp32_scale_differences_pass():
    fp = run(None)
    fp.check(max_bad_frac=0.02)


@pytest.mark.parametrize("bug", ["term", "qd"])
def test_planted_bugs_are_caught(bug):
    fp = run(bug)
    assert fp.unexplained, fp.report()
    with pytest.raises(AssertionError):
        fp.check(max_bad_frac=0.02)
