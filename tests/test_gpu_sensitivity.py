"""GPU: parity gates that resolve 1e-5 (round 4).

The per-env-step tolerances of tests/helpers/forced.py (1e-3 relative) police switching flips; they cannot see a
SYSTEMATIC error of 1e-5..1e-4 (a wrong inertia entry, PD gain or contact constant).  On the random-action Flat
runs a finer gate is not available either: there the oracle moves by ~1e-5 (p50) under a 1e-7 relative perturbation
of the pre-step state (the conditioning probe, ForcedParity.quantiles("cond")), so no fp32 implementation can sit
below that.  These tests put the kernel in well-conditioned states instead (tests/helpers/scenarios.py) and gate
the error QUANTILES of the teacher-forced comparison there (forced.SCEN_GATE, set from the measured fp32 floor);
tests/test_forced_harness.py shows on the CPU that planted 1e-4-relative constant errors move those quantiles past
the gate at the same noise level.

The last test is the north_star criterion (<= 1e-4 relative q error over 1000 policy steps, sim2sim semantics) on a
FREE floating base: zero gravity (no floor contact), so the free joint's quaternion integration and the base row
of the articulated-body solve (M/h12_12dof.xml:68; D/simulator/sim_mujoco.py:39-44,102-121) run for 20 000
substeps next to the fp64 oracle."""
import os

import numpy as np
import pytest
import torch

import oracle as O
from forced import BIAS_GATE, SCEN_GATE, ForcedParity
from h12env import H12FlatEnvCfg, mujoco_cfg
from h12env._abi import F as FIELDS
from h12env.env import H12VelocityEnv
from scenarios import SCENARIOS, SOLE_SCENARIOS, lying_terrain

pytestmark = pytest.mark.gpu

SCALE = dict(flight=1.0, lying=0.3)


def scenario_cfg(task="flat"):
    from h12env.cfg import H12RslEnvCfg

    cfg = H12RslEnvCfg() if task == "rsl" else H12FlatEnvCfg()
    # the lying robots' torso contact is an illegal contact: kept in contact here to measure the contact phase
    cfg.terminations.base_contact_torso = False
    cfg.terminations.base_contact_knees = False
    return cfg


def run_scenario(name, n=1024, steps=20, seed=31, task="flat"):
    cfg = scenario_cfg(task)
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    rng = np.random.default_rng(seed)
    Fm = env._fstate.cpu().numpy().copy()
    SCENARIOS[name](env._model, Fm, rng)
    env._fstate.copy_(torch.from_numpy(Fm))
    fp = ForcedParity(env, seed=seed + 1)
    for _ in range(steps):
        fp.step((rng.normal(size=(n, 12)) * SCALE[name]).astype(np.float32))
    return env, fp


@pytest.mark.parametrize("task", ["flat", "rsl"])
@pytest.mark.parametrize("name", list(SCENARIOS))
def test_forced_error_quantiles_well_conditioned(gpu, name, task):
    """Flat, and the Rsl task (per-env materials and added mass, the 16-term reward table, deadzone commands,
    6-frame history) under its own measured gate (forced.SCEN_GATE[name + "_rsl"])."""
    env, fp = run_scenario(name, task=task)
    fp.check(max_bad_frac=0.01)
    print(name, task, "quantiles", fp.quantiles(), "well-conditioned", fp.quantiles("wc"), "probe",
          fp.quantiles("cond"))
    fp.check_quantiles(SCEN_GATE[name if task == "flat" else name + "_rsl"])
    env.close()


SOLE_KW = dict(stance=dict(preload=1e-3), single_stance={}, slip={})


def run_sole_scenario(name, n=1024, steps=20, seed=37, task="flat"):
    """A sole-contact scenario (tests/helpers/scenarios.py SOLE_SCENARIOS): the state, sole contact flags, anchors and
    action history written into the workspace; the steps driven by the scenario's hold action + N(0, 0.05)."""
    cfg = scenario_cfg(task)
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    rng = np.random.default_rng(seed)
    Fm = env._fstate.cpu().numpy().copy()
    Im = env._istate.cpu().numpy().copy()
    hold = SOLE_SCENARIOS[name](env._model, Fm, rng, Im=Im, action_scale=cfg.actions.joint_pos.scale, **SOLE_KW[name])
    env._fstate.copy_(torch.from_numpy(Fm))
    env._istate.copy_(torch.from_numpy(Im))
    fp = ForcedParity(env, seed=seed + 1)
    for _ in range(steps):
        fp.step((hold + rng.normal(size=(n, 12)) * 0.05).astype(np.float32))
    return env, fp


@pytest.mark.parametrize("task", ["flat", "rsl"])
@pytest.mark.parametrize("name", list(SOLE_SCENARIOS))
def test_forced_sole_contact_scenarios(gpu, name, task):
    """The sole-contact path the benchmark spends its time in (round 5): standing on both feet with the legs'
    stiction springs preloaded, standing on one foot, and both feet slipping (h12_12dof.urdf:168-191 soles,
    V/velocity_env_cfg.py:153-163 material; Rsl: per-env materials).  The depth of a sole contact is the difference
    of ~1 m positions, so fp32 rounding of the state moves the one-step map by ~2e-5 here (the conditioning probe)
    and the absolute-error quantiles cannot resolve 1e-5; the SIGNED mean error per physics-state field does
    (ForcedParity.bias_fields: fp32 rounding averages out over the env-steps, a constant parameter error does not)
    -- forced.BIAS_GATE, per field 6 standard errors + the signed bias of an independent fp32 evaluation of the
    scenario (round 6, tools/gen_sole_bias_gate.py: no term of it is the kernel's own mean), with
    tests/test_forced_harness.py showing on the CPU that planted errors in the stiction spring
    k_t (1e-4), its damper c_t (1e-3), a sole sphere's x offset (1e-4), the normal spring (1e-4) and, slipping, the
    dynamic friction coefficient (1e-4) cross it."""
    env, fp = run_sole_scenario(name, task=task)
    fp.check(max_bad_frac=0.01)
    key = name if task == "flat" else name + "_rsl"
    print(name, task, "quantiles", fp.quantiles(), "probe", fp.quantiles("cond"), "bias", fp.bias())
    if os.environ.get("H12_GATE_MEASURE"):  # calibration runs: report the floors, gate nothing
        import json

        names, m, se = fp.bias_fields()
        out = os.path.join(os.environ["H12_GATE_MEASURE"], f"bias_{key}.json")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        with open(out, "w") as f:
            json.dump({"names": names, "mean": m.tolist(), "se": se.tolist(), "quantiles": fp.quantiles(),
                       "probe": fp.quantiles("cond")}, f)
        env.close()
        pytest.skip("H12_GATE_MEASURE: floors written, nothing gated")
    fp.check_quantiles(SCEN_GATE[key])
    bad = fp.bias_violations(BIAS_GATE[key])
    assert not bad, (bad, fp.bias(), fp.report())
    env.close()


def test_forced_error_quantiles_lying_on_terrain(gpu):
    """The lying scenario on the Rough task's heightfield (C5 randomisation: per-env friction and added torso mass):
    the heightfield contact path (ground_local, the torso face on terrain, the height scan) under the same quantile
    gate as `lying`, forced.SCEN_GATE["lying_terrain"]."""
    from h12env.cfg import c5_cfg

    n = 1024
    cfg = c5_cfg(n)
    cfg.terminations.base_contact_torso = False
    cfg.terminations.base_contact_knees = False
    cfg.sim.device = "cuda:0"
    g = cfg.scene.terrain.terrain_generator
    g.num_rows, g.num_cols, g.border_width = 6, 8, 5.0  # a smaller grid keeps the oracle's terrain setup quick
    env = H12VelocityEnv(cfg)
    t = env.terrain
    O.set_terrain(t.heights, t.hscale, t.x0, t.y0, t.origins)
    env.reset()
    rng = np.random.default_rng(41)
    Fm = env._fstate.cpu().numpy().copy()
    lying_terrain(env._model, Fm, rng, t)
    env._fstate.copy_(torch.from_numpy(Fm))
    fp = ForcedParity(env, seed=42)
    for _ in range(20):
        fp.step((rng.normal(size=(n, 12)) * SCALE["lying"]).astype(np.float32))
    fp.check(max_bad_frac=0.01)
    print("lying_terrain quantiles", fp.quantiles(), "well-conditioned", fp.quantiles("wc"), "probe",
          fp.quantiles("cond"))
    fp.check_quantiles(SCEN_GATE["lying_terrain"])
    env.close()


def test_mujoco_mode_free_base_zero_gravity_1000_steps(gpu, monkeypatch):
    """north_star criterion with the free joint: sim2sim semantics (1 kHz PD, x20 decimation, MJCF clamps, implicit
    joint damping), a floating base in zero gravity (no contact) turned by the legs' reaction, 1000 policy steps of
    random actions: max relative joint-position error <= 1e-4 against the fp64 oracle.  The base orientation is the
    integral of 20 000 substeps of the base's angular velocity; its error is held to 3x the oracle's own divergence
    under a 1e-7 relative state perturbation per policy step (the fp32 conditioning of this trajectory: ~6e-4 rad
    measured; the same probe moves the joints by 1.4e-5..3.3e-5)."""
    import h12env.env as envmod
    from h12env.model import build_model

    def zero_g_model():
        m = build_model()
        m.gravity = 0.0
        return m

    monkeypatch.setattr(envmod, "build_model", zero_g_model)
    n = 8
    cfg = mujoco_cfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = H12VelocityEnv(cfg)
    env.reset()
    assert env._model.gravity == 0.0
    rng = np.random.default_rng(4)
    Fm = env._fstate.cpu().numpy().copy()
    Fm[FIELDS["POS"][0] + 2] = 3.0
    env._fstate.copy_(torch.from_numpy(Fm))
    q0 = np.asarray(env._model.q_default)
    init = [np.concatenate([Fm[o:o + c, i] for o, c in (FIELDS[k] for k in ("POS", "QUAT", "VLIN", "WANG", "Q",
                                                                                "QD"))]).astype(np.float64)
            for i in range(n)]
    steps = 1000
    q_refs = [q0[None] + 0.25 * rng.normal(size=(n, 12)) for _ in range(steps)]

    def oracle_run(eps=0.0):
        prng, S = np.random.default_rng(5), [x.copy() for x in init]
        for t in range(steps):
            for i in range(n):
                x = S[i]
                if eps:  # fp32-scale perturbation of the physics state before every policy step
                    x = x.copy()
                    x[:37] += eps * np.maximum(1.0, np.abs(x[:37])) * prng.choice([-1.0, 1.0], size=37)
                    x[3:7] /= np.linalg.norm(x[3:7])
                S[i], _ = O.mujoco_rollout(env._model, env._ccfg, x, q_refs[t][i].astype(np.float32).astype(np.float64),
                                           20)
        return np.array(S)

    for t in range(steps):
        env.step_physics(torch.from_numpy(q_refs[t].astype(np.float32)).cuda(), 20)
    G = env._fstate.cpu().numpy()
    gs = np.concatenate([G[o:o + c] for o, c in (FIELDS[k] for k in ("POS", "QUAT", "VLIN", "WANG", "Q", "QD"))]).T
    ref, probe = oracle_run(), oracle_run(1e-7)

    def errs(S):
        dq = (np.abs(S[:, 13:25] - ref[:, 13:25]) / np.maximum(1, np.abs(ref[:, 13:25]).max(1, keepdims=True))).max()
        dot = np.abs((S[:, 3:7] * ref[:, 3:7]).sum(axis=1))
        return dq, float(np.max(2 * np.arccos(np.minimum(1.0, dot))))

    (dq, dth), (pq, pth) = errs(gs), errs(probe)
    q_init = np.array(init)[:, 3:7]
    turned = float(np.max(2 * np.arccos(np.minimum(1.0, np.abs((ref[:, 3:7] * q_init).sum(axis=1))))))
    print(f"free base, zero g, 1000 policy steps: GPU max rel q error {dq:.3g}, base orientation error {dth:.3g} rad; "
          f"oracle under 1e-7 perturbations: {pq:.3g}, {pth:.3g} rad; base turned by up to {turned:.3g} rad")
    assert turned > 0.5  # the legs' reaction really turns the base
    assert dq <= 1e-4, (dq, pq)
    assert dth <= 3 * pth, (dth, pth)
    env.close()
