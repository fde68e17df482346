"""The diverged-base termination (round 6): a component of the base's angular velocity above
200 rad/s or of its linear velocity above 50 m/s, or a non-finite one, terminates the episode -- in the oracle
(orc_mdp_terms, CPU) and in the kernel's termination code (through the h12env_eval_terms hook, GPU), the same cases.
No reference counterpart: PhysX does not blow up where the penalty contacts can (profiles/r6/nan_divergence_guard.txt)."""
import numpy as np
import pytest
import torch

import oracle as O
from h12env import H12FlatEnvCfg
from h12env._abi import F as FIELDS

NAN = float("nan")
CASES = [  # (angular velocity, linear velocity, terminated)
    ((0.0, 0.0, 10.0), (1.0, 0.0, 0.0), False),
    ((0.0, 0.0, 199.0), (0.0, 49.0, 0.0), False),
    ((0.0, 0.0, -250.0), (0.0, 0.0, 0.0), True),
    ((0.0, 0.0, 0.0), (60.0, 0.0, 0.0), True),
    ((NAN, 0.0, 0.0), (0.0, 0.0, 0.0), True),
    ((0.0, 0.0, 0.0), (0.0, float("inf"), 0.0), True),
]


def test_oracle_terminates_a_diverged_base(model):
    c = H12FlatEnvCfg().to_c()
    z = np.zeros(12)
    for w, v, want in CASES:
        s = np.zeros(37)
        s[2], s[3] = 1.0, 1.0
        s[7:10], s[10:13] = v, w
        ti = O.term_in(s, z, z, np.zeros(3), np.zeros(2), np.zeros(2), z, z, np.zeros(2), np.zeros(2), 0.0, 1)
        _, term, _ = O.mdp_terms(model, c, ti)
        assert term == want, (w, v)


@pytest.mark.gpu
def test_kernel_terminates_a_diverged_base(gpu):
    from h12env.env import H12VelocityEnv

    n = len(CASES)
    cfg = H12FlatEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    (ow, cw), (ov, cv) = FIELDS["WANG"], FIELDS["VLIN"]
    for i, (w, v, _) in enumerate(CASES):
        env._fstate[ow:ow + cw, i] = torch.tensor(w)
        env._fstate[ov:ov + cv, i] = torch.tensor(v)
    z = torch.zeros(n, 12)
    _, term, _, _ = env.eval_terms(z, z, torch.zeros(n, 5))
    assert term.cpu().tolist() == [c[2] for c in CASES]
    env.close()
