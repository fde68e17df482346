"""GPU: MuJoCo mode (the sim2sim path, row a12) on a FREE-floating base with ground contact, against the CPU oracle.

D/simulator/sim_mujoco.py:39-44,102-121 steps the 12-DoF robot standing on the floor (M/scene_12dof.xml:20) with the
PD law of D/robots/h12_mujoco.py:62-67 at dt = 1 ms x 20 substeps per policy step.  Here the kernel's MuJoCo mode
(h12env_step_physics: PD every substep, MJCF clamps, implicit joint damping, penalty ground contact with anchored
stiction, knee / torso contacts, leg self-collision) is teacher-forced per POLICY step against the oracle's
restatement (oracle/h12_oracle.c, fp64): every step the GPU workspace (state, stiction anchors, contact flags) is
copied into the oracle, both run the same 20 substeps towards the same q_ref, and every env must land within the
harness tolerance (TOL_PHYS relative) or be shown threshold-sensitive by the oracle itself (perturbed re-runs,
tests/helpers/forced.py).  Robots start standing at the default pose, drop onto the floor and are driven by random
joint targets: stance, slip, falls and lying contacts are all reached.  Once with the smooth frictionloss option.
The free-running contact-phase error statistic is tools/mujoco_contact_stats.py."""
import numpy as np
import pytest
import torch

import oracle as O
from forced import TOL_PHYS, phys_err, unexplained_envs
from h12env import mujoco_cfg
from h12env._abi import I as IFIELDS
from h12env.env import H12VelocityEnv

pytestmark = pytest.mark.gpu


def contact_envs(I):
    pack = I[IFIELDS["PACK"][0]]
    return ((pack >> 13) & 0xFF) != 0


@pytest.mark.parametrize("frictionloss", [False, True])
def test_mujoco_mode_free_base_contact_teacher_forced(gpu, frictionloss):
    n, steps = 128, 150
    cfg = mujoco_cfg()
    cfg.sim.frictionloss = frictionloss
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    ref = O.OracleEnv(env._model, env._ccfg, n)
    rng = np.random.default_rng(11)
    q0 = np.asarray(env._model.q_default, np.float32)
    bad_total = off_total = in_contact = 0
    for t in range(steps):
        F0 = env._fstate.cpu().numpy().copy()
        I0 = env._istate.cpu().numpy().copy()
        q_ref = (q0[None] + 0.25 * 0.6 * rng.normal(size=(n, 12))).astype(np.float32)
        env.step_physics(torch.from_numpy(q_ref).cuda(), 20)
        g = env._fstate.cpu().numpy().copy()
        gi = env._istate.cpu().numpy().copy()

        def rerun(Fp):
            ref.F[:], ref.I[:] = Fp, I0
            ref.step_physics(q_ref, 20)
            return ref.F.copy()

        o = rerun(F0)
        oi = ref.I.copy()
        assert np.isfinite(g).all()
        gerr = phys_err(g, o) / TOL_PHYS
        err = lambda a, b: phys_err(a, b) / TOL_PHYS  # noqa: E731
        bad = unexplained_envs(F0, gerr, 1.0, rerun, err, o, g, seed=t)
        assert bad.size == 0, (t, bad[:8], gerr[bad[:8]])
        off_total += int((gerr > 1.0).sum())
        in_contact += int(contact_envs(oi).sum())
        # contact flags of the sole spheres: identical wherever the state is within tolerance
        ok = gerr <= 1.0
        assert (contact_envs(gi)[ok] == contact_envs(oi)[ok]).mean() > 0.99
    frac_contact = in_contact / (n * steps)
    print(f"frictionloss={frictionloss}: env-steps off tolerance {off_total} of {n * steps} (all threshold-sensitive); "
          f"sole contact in {frac_contact:.2f} of env-steps")
    assert frac_contact > 0.3  # a contact phase, not free flight
    assert off_total <= 0.02 * n * steps
    env.close()
