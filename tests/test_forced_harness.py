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
from forced import SCEN_GATE, ForcedParity, perturbed
from h12env import H12FlatEnvCfg
from h12env._abi import F as FIELDS
from h12env.model import build_model


class OracleStandIn:
    """The surface ForcedParity drives (H12VelocityEnv's), backed by the CPU oracle."""

    def __init__(self, n, bug=None, seed=0, cfg=None, noise=1e-7):
        cfg = cfg or H12FlatEnvCfg()
        cfg.scene.num_envs = n
        self._model, self._ccfg = build_model(), cfg.to_c()  # what the harness's oracle runs
        self.num_envs, self.env_offset, self.device = n, 0, torch.device("cpu")
        model, ccfg = build_model(), cfg.to_c()  # what the stand-in runs (a planted constant error below)
        name, rel = (bug.split(":")[0], float(bug.split(":")[1])) if bug and ":" in bug else (bug, 1e-4)
        if name == "inertia":  # one link's rotational inertia (left knee, all six entries) too large
            for k in range(6):
                model.link_inertia[3][k] *= 1.0 + rel
        elif name == "kd":  # the PD damping gain of one joint (left hip pitch) too large
            ccfg.kd[0] *= 1.0 + rel
        elif name == "contact_c":  # the ground-contact damper too large
            ccfg.contact_c *= 1.0 + rel
        elif name == "contact_k":  # the ground-contact spring too large
            ccfg.contact_k *= 1.0 + rel
        elif name == "mass":  # one link's mass (left ankle pitch) too large
            model.link_mass[4] *= 1.0 + rel
        elif name == "friction_k":  # the sole stiction spring k_t too large
            ccfg.friction_k *= 1.0 + rel
        elif name == "friction_c":  # the sole stiction damper c_t too large
            ccfg.friction_c *= 1.0 + rel
        elif name == "sole_x":  # one sole sphere's x offset (the heel's, foot frame) too large
            model.foot_pts[0][0] *= 1.0 + rel
        elif name == "mu_d":  # the dynamic (slipping) friction coefficient too SMALL
            ccfg.mu_dynamic *= 1.0 - rel
        elif name == "mu_s":  # the static (stick / slip) friction coefficient too SMALL
            ccfg.mu_static *= 1.0 - rel
        elif name == "gravity":  # gravity too strong (the sole gate's force-balance allowance, gen_sole_bias_gate.py)
            model.gravity *= 1.0 + rel
        self.core = O.OracleEnv(model, ccfg, n)
        if cfg.scene.terrain.terrain_type == "generator":  # startup state (origins, materials) and the heightfield
            from h12env.startup import apply_to_arrays, startup_state

            st = startup_state(cfg, n)
            apply_to_arrays(st, self.core.F, self.core.I)
            t = st.terrain
            O.set_terrain(t.heights, t.hscale, t.x0, t.y0, t.origins)
            self.terrain = t
        self.core.reset()
        self._fstate = torch.from_numpy(self.core.F)
        self._istate = torch.from_numpy(self.core.I)
        self._obs = [torch.from_numpy(self.core.obs)]
        self._k = 0
        self.common_step_counter = 0
        self.bug, self.noise = bug, noise
        self.rng = np.random.default_rng(seed)

    def step(self, a):
        self.common_step_counter += 1
        self.core.F[:] = perturbed(self.rng, self.core.F, self.noise)  # fp32-scale "rounding" of the stand-in
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


def run(bug, n=64, steps=25, scale=1.0):
    env = OracleStandIn(n, bug)
    fp = ForcedParity(env, seed=1)
    rng = np.random.default_rng(2)
    for _ in range(steps):
        fp.step((rng.normal(size=(n, 12)) * scale).astype(np.float32))
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


# Constant-parameter errors of 1e-4 relative stay far inside the per-env-step tolerances (1e-3) but shift the bulk
# of the error distribution in the well-conditioned scenarios (tests/helpers/scenarios.py): the scenario quantile
# gates (forced.SCEN_GATE, the ones tests/test_gpu_sensitivity.py applies to the kernel) must pass the clean stand-in
# and reject each planted error.  The stand-in's rounding noise is calibrated to the GPU's measured floor in each
# scenario (clean p50 of the phys error at least the kernel's: flight 1.37e-6, lying 2.64e-6 -- DESIGN.md section 4),
# so what is caught here is caught at the kernel's own noise level.  The contact damper (c = 100 N s/m carries ~1 %
# of the contact force at these speeds) is planted at 1e-3: a 1e-4 error in it moves the state by ~1e-6 relative,
# under that floor.  The link mass is caught in flight (its effect in the contact phase is below the floor there).
SCEN_NOISE = dict(flight=5e-8, lying=4e-8)
SCEN_SCALE = dict(flight=1.0, lying=0.3)
SCEN_BUGS = dict(flight=("inertia", "kd", "mass"), lying=("inertia", "kd", "contact_k", "contact_c:1e-3"))


def run_scenario(name, bug, n=128, steps=20):
    from h12env import H12FlatEnvCfg
    from scenarios import SCENARIOS

    cfg = H12FlatEnvCfg()
    cfg.terminations.base_contact_torso = False
    cfg.terminations.base_contact_knees = False
    env = OracleStandIn(n, bug, cfg=cfg, noise=SCEN_NOISE[name])
    SCENARIOS[name](env._model, env.core.F, np.random.default_rng(5))
    fp = ForcedParity(env, seed=1)
    rng = np.random.default_rng(2)
    for _ in range(steps):
        fp.step((rng.normal(size=(n, 12)) * SCEN_SCALE[name]).astype(np.float32))
    return fp


@pytest.mark.parametrize("name", list(SCEN_BUGS))
def test_scenario_gate_passes_clean_stand_in(name):
    fp = run_scenario(name, None)
    fp.check(max_bad_frac=0.02)
    fp.check_quantiles(SCEN_GATE[name])


@pytest.mark.parametrize("name,bug", [(k, b) for k, v in SCEN_BUGS.items() for b in v])
def test_scenario_gate_catches_small_constant_errors(name, bug):
    fp = run_scenario(name, bug)
    assert fp.quantile_violations(SCEN_GATE[name]), fp.report()


# The heightfield lying scenario (C5 randomisation) under forced.SCEN_GATE["lying_terrain"]: stand-in noise calibrated
# to the kernel's floor there (clean p50 of the phys error >= 5.2e-6), planted 1e-4 constant errors caught.
TERRAIN_NOISE = 4e-8  # clean p50 5.0e-6 against the kernel's 5.2e-6


def run_terrain(bug, n=96, steps=16):
    from h12env.cfg import c5_cfg
    from scenarios import lying_terrain

    cfg = c5_cfg(n)
    cfg.terminations.base_contact_torso = False
    cfg.terminations.base_contact_knees = False
    g = cfg.scene.terrain.terrain_generator
    g.num_rows, g.num_cols, g.border_width = 6, 8, 5.0
    env = OracleStandIn(n, bug, cfg=cfg, noise=TERRAIN_NOISE)
    lying_terrain(env._model, env.core.F, np.random.default_rng(5), env.terrain)
    fp = ForcedParity(env, seed=1)
    rng = np.random.default_rng(2)
    for _ in range(steps):
        fp.step((rng.normal(size=(n, 12)) * SCEN_SCALE["lying"]).astype(np.float32))
    return fp


def test_terrain_gate_passes_clean_stand_in():
    fp = run_terrain(None)
    fp.check(max_bad_frac=0.02)
    fp.check_quantiles(SCEN_GATE["lying_terrain"])


@pytest.mark.parametrize("bug", ["inertia", "kd", "contact_k"])
def test_terrain_gate_catches_small_constant_errors(bug):
    fp = run_terrain(bug)
    assert fp.quantile_violations(SCEN_GATE["lying_terrain"]), fp.report()


# The sole-contact scenarios (round 5; forced.BIAS_GATE, tests/golden/sole_bias_gate.json).  Their absolute-error
# quantiles sit at the fp32 floor of a sole depth computed from ~1 m positions (the kernel's p50 5.5e-5 against the
# oracle's own conditioning probe 3.8e-5), so a constant 1e-4 error in the tangential contact shows up in the SIGNED
# mean error per physics-state field instead.  The stand-in's rounding noise is calibrated to the kernel's floor there
# (clean p50 of the phys error >= the kernel's 5.2-6.2e-5); the gate (3x the kernel's own per-field fp32 bias + 6 of
# its standard errors) must pass the clean stand-in and reject: the stiction spring k_t +1e-4, its damper c_t +1e-3
# (c_t carries little of a sticking sole's force: like the normal damper, caught at 1e-3), one sole sphere's x offset
# +1e-4 relative (8 um), the normal spring +1e-4 and, slipping, the dynamic friction coefficient -1e-4.  mu_s is a
# pure switching threshold in this contact law (stick while |f_t| <= mu_s f_n; a slipping sole is dragged at mu_d f_n,
# oracle contact_point): an error in it moves only the decisions of contacts within that relative distance of the
# cap, and a slipping sole's decision 1e-4 from the cap is within the fp32 resolution of its anchor offset (~3e-5 of
# a 2 mm offset at ~0.1 m positions) -- it cannot be told from rounding (the clean and mu_s:1e-4 slip runs are
# identical: every sole there is far above the cap).
SOLE_NOISE = 1.5e-7
SOLE_BUGS = dict(stance=("friction_k", "sole_x"),
                 single_stance=("friction_k", "friction_c:1e-3", "sole_x", "contact_k", "mu_d"),
                 slip=("friction_k", "sole_x", "contact_k", "mu_d"))


def run_sole(name, bug, n=1024, steps=20):
    from h12env import H12FlatEnvCfg
    from scenarios import SOLE_SCENARIOS

    cfg = H12FlatEnvCfg()
    cfg.terminations.base_contact_torso = False
    cfg.terminations.base_contact_knees = False
    env = OracleStandIn(n, bug, cfg=cfg, noise=SOLE_NOISE)
    kw = dict(preload=1e-3) if name == "stance" else {}
    hold = SOLE_SCENARIOS[name](env._model, env.core.F, np.random.default_rng(5), Im=env.core.I, action_scale=0.5,
                                **kw)
    fp = ForcedParity(env, seed=1)
    rng = np.random.default_rng(2)
    for _ in range(steps):
        fp.step((hold + rng.normal(size=(n, 12)) * 0.05).astype(np.float32))
    return fp


@pytest.mark.parametrize("name", list(SOLE_BUGS))
def test_sole_gate_passes_clean_stand_in(name):
    from forced import BIAS_GATE

    fp = run_sole(name, None)
    fp.check(max_bad_frac=0.02)
    q = fp.quantiles()["phys"]["p50"]
    assert q >= 0.8 * min(v["phys"][0] for k, v in SCEN_GATE.items() if k.startswith(name)) / 2, q  # noise at the floor
    assert not fp.bias_violations(BIAS_GATE[name]), fp.bias()


@pytest.mark.parametrize("name,bug", [(k, b) for k, v in SOLE_BUGS.items() for b in v])
def test_sole_gate_catches_tangential_contact_errors(name, bug):
    from forced import BIAS_GATE

    fp = run_sole(name, bug)
    assert fp.bias_violations(BIAS_GATE[name]), fp.bias()
