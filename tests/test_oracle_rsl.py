"""CPU: the Rsl task (row f4, Isaac-Velocity-Rsl-H12_12dof-v0, rsl_env_cfg.py) -- its cfg -> C-ABI mapping,
the deploy env.yaml it exports (pinned EXACTLY by the shipped scripts/deploy/policies/{demo_rsl,success_1,
success_2}/env.yaml, which were exported from this task), and the oracle's restatement of its MDP
additions: the 270-float observation (history 6, ang_vel x 0.25, joint_vel x 0.05 after noise), the deadzone
command (utils/mdp/commands.py:41-96), the push interval event, and the extra reward terms.

Parity of the physics / managers against IsaacLab itself is unpinned (not installed); these tests pin the
oracle's semantics, which the GPU tests then hold the kernel to."""
import json
from pathlib import Path

import numpy as np
import pytest
import yaml

import oracle as O
from h12env._abi import F as FIELDS
from h12env._abi import NREW, REWARD_FUNCS
from h12env.cfg import H12FlatEnvCfg, H12RslEnvCfg, H12RslEnvCfg_PLAY, RewTerm
from h12env.export import deploy_config, write_env_yaml

GOLD = Path(__file__).resolve().parent / "golden"
RID = {f: i for i, f in enumerate(REWARD_FUNCS)}


def test_rsl_cfg_maps_onto_the_kernel_terms():
    cfg = H12RslEnvCfg()
    c = cfg.to_c()
    w = np.array(c.rew_w)
    want = {"track_lin_vel_xy_exp": 1.0, "track_ang_vel_z_exp": 0.5, "feet_air_time_positive_biped": 0.75,
            "feet_slide": -0.25, "flat_orientation_l2": -1.0, "base_height_l2": -0.2, "joint_torques_l2": -1e-5,
            "joint_vel_l2": -1e-3, "joint_acc_l2": -1e-7, "joint_deviation_l1:hip": -0.2,
            "joint_deviation_l1:ankle": -0.2, "joint_pos_limits:ankle": -0.2, "joint_pos_limits:hip": -0.2,
            "action_rate_l2": -0.01, "contact_forces": -1e-3, "is_terminated": -200.0}
    got = {REWARD_FUNCS[i]: float(w[i]) for i in range(NREW) if w[i] != 0}
    assert got.keys() == want.keys()
    for k, v in want.items():
        assert got[k] == pytest.approx(v, rel=1e-6), k
    # the 16 terms keep the cfg's RewardManager order for the log
    assert [k for k, _ in cfg.rewards.active()][:3] == ["track_lin_vel_xy_exp", "track_ang_vel_z_exp", "feet_air_time"]
    assert len(cfg.rewards.active()) == 16
    assert c.base_height_target == pytest.approx(1.0) and c.contact_force_threshold == pytest.approx(800.0)
    # IdealPD: no delay; action scale 0.25; deadzone commands over U(5, 8) s with +-1 ranges, no heading
    assert (c.min_delay, c.max_delay) == (0, 0) and c.action_scale == pytest.approx(0.25)
    assert c.cmd_deadzone == 1 and c.velocity_deadzone == 0.0
    assert (c.cmd_resample_time, c.cmd_resample_time_max) == (5.0, 8.0)
    assert c.ang_flip_prob == pytest.approx(0.005 / 20.0)
    assert c.rel_heading_envs < 0
    assert list(c.cmd_lin_x) == [-1, 1] and list(c.cmd_lin_y) == [-1, 1] and list(c.cmd_ang_z) == [-1, 1]
    assert c.history_length == 6 and list(np.round(c.obs_scale, 6)) == [0.25, 1, 1, 1, 0.05, 1]
    assert c.push_enable == 1 and list(c.push_interval) == [5, 8] and list(c.push_vel_x) == [-1, 1]
    assert c.per_env_friction == 1 and c.per_env_mass == 0
    assert len(cfg.curriculum.reward_weights) == 12
    assert all(t.num_steps == 24 * 5000 for t in cfg.curriculum.reward_weights)
    p = H12RslEnvCfg_PLAY().to_c()
    assert p.push_enable == 0 and p.per_env_friction == 0 and p.enable_corruption == 0
    assert p.mu_static == pytest.approx(1.0) and list(p.cmd_lin_x) == [0.5, 0.5]


def test_reward_terms_validate():
    cfg = H12FlatEnvCfg()
    cfg.rewards.lin_vel_z_l2 = RewTerm(-2.0, func="lin_vel_z_l2")
    assert cfg.to_c().rew_w[RID["lin_vel_z_l2"]] == pytest.approx(-2.0)
    cfg.rewards.lin_vel_z_l2 = None                       # removed, as IsaacLab's `= None`
    assert cfg.to_c().rew_w[RID["lin_vel_z_l2"]] == 0.0
    with pytest.raises(AttributeError):
        cfg.rewards.undesired_contacts = RewTerm(-1.0)    # no kernel term
    cfg.rewards.dup = RewTerm(-1.0, func="ang_vel_xy_l2")
    with pytest.raises(ValueError):
        cfg.to_c()


def test_rsl_env_yaml_equals_the_shipped_deploy_configs(tmp_path):
    """get_deploy_config(Rsl task) must reproduce scripts/deploy/policies/{demo_rsl,success_1,success_2}/env.yaml."""
    ref = json.loads((GOLD / "deploy_env_yaml.json").read_text())
    d = yaml.safe_load(open(write_env_yaml(H12RslEnvCfg(), str(tmp_path / "env.yaml"))))
    for name in ("demo_rsl", "success_1", "success_2"):
        r = ref[name]
        assert list(d.keys()) == r["keys"], name
        assert d["observations"] == r["observations"], name
        for k in ("history_length", "action_scale", "velocity_deadzone", "history_step"):
            assert d[k] == r[k], (name, k)
        assert d["control_dt"] == pytest.approx(r["control_dt"])
        assert d["command_ranges"] == r["command_ranges"], name
        assert [{k: j[k] for k in ("name", "kp", "kd", "enabled")} for j in d["joints"]] == \
               [{k: j[k] for k in ("name", "kp", "kd", "enabled")} for j in r["leg_joints"]]
        np.testing.assert_allclose([j["default_joint_pos"] for j in d["joints"]],
                                   [j["default_joint_pos"] for j in r["leg_joints"]], atol=1e-9)
    assert deploy_config(H12RslEnvCfg_PLAY())["command_ranges"]["lin_vel_x"] == [0.5, 0.5]


def rsl_oracle(model, n, **kw):
    cfg = H12RslEnvCfg()
    cfg.scene.num_envs = n
    for k, v in kw.items():
        setattr(cfg, k, v)
    from h12env.startup import apply_to_arrays, startup_state

    c = cfg.to_c()
    env = O.OracleEnv(model, c, n)
    apply_to_arrays(startup_state(cfg, n), env.F, env.I)
    O.set_dz_count(0)
    return env, cfg, c


def test_rsl_observation_layout_history_and_scales(model):
    n = 8
    env, cfg, c = rsl_oracle(model, n)
    c.enable_corruption = 0
    env.cfg = c
    obs = env.reset()
    assert obs.shape == (n, 270)
    F = env.F
    # term-major blocks of 6 frames: ang_vel (18), gravity (18), command (18), q (72), qd (72), action (72)
    w = F[FIELDS["WANG"][0]:FIELDS["WANG"][0] + 3].T
    cmd = F[FIELDS["CMD"][0]:FIELDS["CMD"][0] + 3].T
    for h in range(6):
        np.testing.assert_allclose(obs[:, 3 * h:3 * h + 3], 0.25 * w, atol=1e-7)
        np.testing.assert_allclose(obs[:, 36 + 3 * h:36 + 3 * h + 3], cmd, atol=1e-7)
    # after a step with large random actions the newest frame differs from the older ones; qd x 0.05
    rng = np.random.default_rng(0)
    obs1, *_ = env.step(rng.normal(size=(n, 12)).astype(np.float32), 1)
    qd = env.F[FIELDS["QD"][0]:FIELDS["QD"][0] + 12].T
    np.testing.assert_allclose(obs1[:, 126 + 60:126 + 72], 0.05 * qd, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(obs1[:, 126:126 + 60], obs[:, 126 + 12:126 + 72], atol=0)   # shifted history


def test_deadzone_commands_and_flips(model):
    n = 2048
    env, cfg, c = rsl_oracle(model, n)
    env.reset()
    cmd0 = env.F[FIELDS["CMD"][0]:FIELDS["CMD"][0] + 3].copy()
    assert (np.abs(cmd0[:2]).sum(axis=0) > 0).all()          # fresh U(-1, 1) commands, no standing zeroing
    env.step(np.zeros((n, 12), np.float32), 1)
    cmd1 = env.F[FIELDS["CMD"][0]:FIELDS["CMD"][0] + 3]
    zeroed = (cmd1[0] == 0) & (cmd1[1] == 0)
    # velocity_deadzone 0: every step each env's xy command is zeroed with probability 1/2
    assert abs(zeroed.mean() - 0.5) < 5 * np.sqrt(0.25 / n)
    np.testing.assert_array_equal(cmd1[:2, ~zeroed], cmd0[:2, ~zeroed])
    assert O.dz_count() == 0                                  # |cmd| < 0 never holds
    # angular-velocity sign flips at the configured rate
    c.ang_flip_prob = 0.25
    env.cfg = c
    before = env.F[FIELDS["CMD"][0] + 2].copy()
    env.step(np.zeros((n, 12), np.float32), 2)
    flipped = env.F[FIELDS["CMD"][0] + 2] == -before
    assert abs(flipped.mean() - 0.25) < 5 * np.sqrt(0.25 * 0.75 / n)
    # a positive deadzone: the count carried to the next step is the number of envs inside it
    c.velocity_deadzone = 0.5
    env.cfg = c
    env.step(np.zeros((n, 12), np.float32), 3)
    cm = env.F[FIELDS["CMD"][0]:FIELDS["CMD"][0] + 2]
    assert O.dz_count() == int(((cm[0].astype(np.float32) ** 2 + cm[1] ** 2) < np.float32(0.25)).sum())


def test_push_event_interval_and_velocity(model):
    n = 256
    env, cfg, c = rsl_oracle(model, n)
    env.reset()
    pt = env.F[FIELDS["PUSH_TIME"][0]]
    assert (pt >= 5.0).all() and (pt <= 8.0).all()
    # put every env 1 step from its push and compare with the same step without the push
    env.F[FIELDS["PUSH_TIME"][0]] = 0.01
    F0, I0 = env.F.copy(), env.I.copy()
    c2 = H12RslEnvCfg()
    c2.events.push_robot = None
    ref = O.OracleEnv(model, c2.to_c(), n)
    ref.F[:], ref.I[:] = F0, I0
    ref.obs[:] = env.obs
    env.step(np.zeros((n, 12), np.float32), 1)
    ref.step(np.zeros((n, 12), np.float32), 1)
    v, vr = env.F[FIELDS["VLIN"][0]:FIELDS["VLIN"][0] + 3], ref.F[FIELDS["VLIN"][0]:FIELDS["VLIN"][0] + 3]
    dv = v - vr
    assert (np.abs(dv[:2]) <= 1.0 + 1e-6).all() and np.abs(dv[:2]).mean() > 0.3
    np.testing.assert_allclose(dv[2], 0, atol=1e-7)
    pt = env.F[FIELDS["PUSH_TIME"][0]]
    assert (pt >= 5.0 - 1e-6).all() and (pt <= 8.0).all()


def test_rsl_reward_terms_by_isolation(model):
    """Weight one term at a time and compare the reward with the term recomputed from the post-step state."""
    n = 64
    rng = np.random.default_rng(5)
    a = (0.3 * rng.normal(size=(n, 12))).astype(np.float32)
    q0 = np.asarray(model.q_default)
    lo, hi = np.asarray(model.q_lower), np.asarray(model.q_upper)
    mid, half = (lo + hi) / 2, (hi - lo) / 2 * 0.9
    checks = {
        "base_height_l2": lambda F: (F[FIELDS["POS"][0] + 2] - 1.0) ** 2,
        "joint_vel_l2": lambda F: (F[FIELDS["QD"][0]:FIELDS["QD"][0] + 12] ** 2).sum(0),
        "joint_deviation_l1:ankle": lambda F: np.abs(F[FIELDS["Q"][0]:FIELDS["Q"][0] + 12] - q0[:, None])[[4, 5, 10, 11]].sum(0),
        "joint_pos_limits:hip": lambda F: (np.clip((mid - half)[:, None] - F[FIELDS["Q"][0]:FIELDS["Q"][0] + 12], 0, None)
                                           + np.clip(F[FIELDS["Q"][0]:FIELDS["Q"][0] + 12] - (mid + half)[:, None], 0, None))[[0, 2, 6, 8]].sum(0),
        "track_ang_vel_z_exp": lambda F: np.exp(-(F[FIELDS["CMD"][0] + 2] - F[FIELDS["WANG"][0] + 2]) ** 2 / 0.25),
    }
    for func, want_fn in checks.items():
        env, cfg, c = rsl_oracle(model, n)
        for t in range(NREW):
            c.rew_w[t] = 0.0
        c.rew_w[RID[func]] = 1.0
        c.cmd_deadzone = 0                    # keep the command fixed across the step
        c.push_enable = 0
        c.cmd_resample_time = c.cmd_resample_time_max = 100.0
        c.rel_standing_envs = -1.0            # standing envs would zero the command after the reward
        env.cfg = c
        env.reset()
        aa = a.copy()
        if func == "joint_pos_limits:hip":   # drive the hip yaws past their soft limits (+-0.387)
            aa[:, 0], aa[:, 6] = 6.0, -6.0
        _, rew, term, trunc, _ = env.step(aa, 1)
        ok = ~(term | trunc)
        want = want_fn(env.F) * 0.02
        np.testing.assert_allclose(rew[ok], want[ok], rtol=2e-5, atol=1e-8, err_msg=func)
        if func == "joint_pos_limits:hip":
            assert (want[ok] > 0).any()
