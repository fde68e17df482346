"""CPU: the oracle's rough-task restatement (row f2) -- heightfield ground, contact on it, the 235-float
observation with the height scan, terrain curriculum, per-env friction / added torso mass.

Parity against IsaacLab's terrain generator / PhysX is unpinned (neither is installed); these tests pin
the oracle's own semantics: the ground query equals the host twin of the mesh interpolation, resets place
robots on their sub-terrain origin, the scan reads the terrain under a known pose, the curriculum moves
levels exactly as terrain_levels_vel specifies, and the added mass shows up in the mass matrix.
"""
import numpy as np
import pytest

import oracle as O
from h12env import terrain as T
from h12env._abi import F as FIELDS
from h12env._abi import I as IFIELDS
from h12env._abi import NOBS_ROUGH
from h12env.cfg import H12RoughEnvCfg, c5_cfg
from h12env.startup import apply_to_arrays, startup_state


def small_rough(n=16, **kw):
    cfg = H12RoughEnvCfg()
    cfg.scene.num_envs = n
    g = cfg.scene.terrain.terrain_generator
    g.num_rows, g.num_cols, g.border_width = 4, 4, 4.0
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def oracle_env(model, cfg, n):
    st = startup_state(cfg, n)
    O.set_terrain(st.terrain.heights, st.terrain.hscale, st.terrain.x0, st.terrain.y0, st.terrain.origins)
    env = O.OracleEnv(model, cfg.to_c(), n)
    apply_to_arrays(st, env.F, env.I)
    return env, st


def test_ground_matches_host_mesh_twin():
    cfg = small_rough()
    t = T.generate(cfg.scene.terrain.terrain_generator, 3)
    O.set_terrain(t.heights, t.hscale, t.x0, t.y0, t.origins)
    c = cfg.to_c()
    rng = np.random.default_rng(0)
    xs = rng.uniform(t.x0 - 1, t.x0 + t.hscale * t.shape[0] + 1, 500)
    ys = rng.uniform(t.y0 - 1, t.y0 + t.hscale * t.shape[1] + 1, 500)
    want = T.ground_height(t, xs, ys)
    got = np.array([O.ground(c, x, y)[0] for x, y in zip(xs, ys)])
    np.testing.assert_allclose(got, want, atol=1e-9)
    # vertices are exact, heights are multiples of the vertical scale within the noise range
    assert t.heights.min() >= 0 and t.heights.max() <= 0.02 + 1e-7
    np.testing.assert_allclose(np.round(t.heights / 0.005) * 0.005, t.heights, atol=1e-7)
    # slope of a triangle from finite differences
    h, gx, gy = O.ground(c, 1.234, -0.567)
    e = 1e-6
    hx = (O.ground(c, 1.234 + e, -0.567)[0] - O.ground(c, 1.234 - e, -0.567)[0]) / (2 * e)
    assert gx == pytest.approx(hx, abs=1e-4)


def test_reset_on_origins_and_obs_layout(model):
    n = 16
    cfg = small_rough(n)
    env, st = oracle_env(model, cfg, n)
    obs = env.reset()
    assert obs.shape == (n, NOBS_ROUGH)
    org = st.fields["ORIGIN"]
    pos = env.F[FIELDS["POS"][0]:FIELDS["POS"][0] + 3]
    assert (np.abs(pos[0:2] - org[0:2]) <= 0.5 + 1e-6).all()
    np.testing.assert_allclose(pos[2], org[2] + 1.05, atol=1e-6)
    # height scan ~ sensor z - ground - 0.5 = 0.55 + origin_z - ground (+- 0.1 noise), clipped to +-1
    scan = obs[:, 48:]
    assert (np.abs(scan) <= 1.0).all()
    assert np.abs(scan.mean() - 0.55) < 0.05
    # base_lin_vel / ang_vel are zero-mean noise at reset, gravity ~ (0, 0, -1)
    np.testing.assert_allclose(obs[:, 6:9].mean(axis=0), [0, 0, -1], atol=0.03)


def test_noise_free_scan_reads_terrain(model):
    n = 4
    cfg = small_rough(n)
    cfg.observations.policy.enable_corruption = False
    env, st = oracle_env(model, cfg, n)
    obs = env.reset()
    c = cfg.to_c()
    t = st.terrain
    p = env.F[FIELDS["POS"][0]:FIELDS["POS"][0] + 3, 0]
    qw, qz = env.F[FIELDS["QUAT"][0], 0], env.F[FIELDS["QUAT"][0] + 3, 0]
    yaw = 2 * np.arctan2(qz, qw)
    k = 0
    for iy in range(11):
        for ix in range(17):
            xl, yl = 0.1 * (ix - 8), 0.1 * (iy - 5)
            x = p[0] + np.cos(yaw) * xl - np.sin(yaw) * yl
            y = p[1] + np.sin(yaw) * xl + np.cos(yaw) * yl
            want = np.clip(p[2] - T.ground_height(t, np.array([x]), np.array([y]))[0] - 0.5, -1, 1)
            assert obs[0, 48 + k] == pytest.approx(want, abs=2e-5)
            k += 1
    del c


def test_curriculum_levels(model):
    n = 3
    cfg = small_rough(n)
    env, st = oracle_env(model, cfg, n)
    env.reset()
    I0 = IFIELDS["TERRAIN"][0]
    o, p = FIELDS["ORIGIN"][0], FIELDS["POS"][0]
    cmd = FIELDS["CMD"][0]
    env.I[I0] = np.array([1, 2, 3]) | (np.array([0, 1, 2]) << 16)
    org = st.terrain.origins
    for i, (lv, ty) in enumerate([(1, 0), (2, 1), (3, 2)]):
        env.F[o:o + 3, i] = org[lv, ty]
    # env 0 walked 5 m (> 8/2): up; env 1 stood still with a 1 m/s command: down; env 2 at the last
    # level walked far: random level
    env.F[p:p + 2, 0] = org[1, 0, :2] + np.array([5.0, 0.0])
    env.F[p:p + 2, 1] = org[2, 1, :2]
    env.F[cmd, 1] = 1.0
    env.F[p:p + 2, 2] = org[3, 2, :2] + np.array([0.0, 4.5])
    env.reset()
    lv = env.I[I0] & 0xFFFF
    ty = env.I[I0] >> 16
    assert lv[0] == 2 and lv[1] == 1 and 0 <= lv[2] < 4
    assert list(ty) == [0, 1, 2]
    for i in range(3):
        np.testing.assert_allclose(env.F[o:o + 3, i], org[lv[i], ty[i]])


def test_added_mass_in_mass_matrix_and_friction_buckets(model):
    n = 64
    cfg = c5_cfg(n)
    st = startup_state(cfg, n)
    mu = st.fields["MU"]
    assert mu.shape == (4, n) and (mu >= 0.1 - 1e-6).all() and (mu <= 1.25 + 1e-6).all()
    assert len(np.unique(mu[0])) <= 64
    dm = st.fields["DMASS"][0]
    assert (dm >= 0).all() and (dm <= 6).all()
    p = O.Phys()
    p.quat[0] = 1.0
    p.pos[2] = 2.0
    p.env_params = 1
    p.dmass = 4.0
    M = np.zeros((18, 18))
    import ctypes as C
    O.lib().orc_mass_matrix(C.byref(model), C.byref(p), M.ctypes.data_as(C.POINTER(C.c_double)))
    np.testing.assert_allclose(np.diag(M)[3:6], [67.3676 + 4.0] * 3, atol=1e-3)


def test_rough_standing_is_stable(model):
    """Default-pose PD on the heightfield: the robot stands for 1 s (no fall, bounded slip)."""
    n = 8
    cfg = small_rough(n)
    env, _ = oracle_env(model, cfg, n)
    env.reset()
    z0 = env.F[FIELDS["POS"][0] + 2].copy()
    for t in range(50):
        obs, rew, term, trunc, _ = env.step(np.zeros((n, 12), np.float32), t + 1)
        assert not term.any()
    z1 = env.F[FIELDS["POS"][0] + 2]
    assert (np.abs(z1 - z0) < 0.15).all()
