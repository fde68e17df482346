"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
The product path (h12env -> libh12env.so) never does.
"""
from __future__ import annotations

import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))

from h12env._abi import NF_FLOAT, NF_INT, NJ, NLOG, NOBS, H12Config, H12Model  # noqa: E402

LIB = HERE / "liboracle.so"


class Phys(C.Structure):
    _fields_ = [("pos", C.c_double * 3), ("quat", C.c_double * 4), ("vlin", C.c_double * 3),
                ("wang", C.c_double * 3), ("q", C.c_double * NJ), ("qd", C.c_double * NJ),
                ("anchor", C.c_double * 16), ("cmask", C.c_int32), ("env_params", C.c_int32),
                ("mu", C.c_double * 4), ("dmass", C.c_double)]

    def to_numpy(self) -> np.ndarray:
        """37 physics coordinates + 16 anchors + contact mask (as float)."""
        return np.concatenate([np.array(self.pos), np.array(self.quat), np.array(self.vlin), np.array(self.wang),
                               np.array(self.q), np.array(self.qd), np.array(self.anchor), [float(self.cmask)]])

    @classmethod
    def from_numpy(cls, x) -> "Phys":
        x = np.asarray(x, dtype=np.float64)
        p = cls()
        p.pos[:] = x[0:3]
        p.quat[:] = x[3:7]
        p.vlin[:] = x[7:10]
        p.wang[:] = x[10:13]
        p.q[:] = x[13:25]
        p.qd[:] = x[25:37]
        if x.size >= 54:
            p.anchor[:] = x[37:53]
            p.cmask = int(x[53])
        return p


class TermIn(C.Structure):
    """orc_term_in: the post-physics snapshot the MDP terms / CaT constraints are evaluated on."""
    _fields_ = [("p", Phys), ("act", C.c_double * NJ), ("act_prev", C.c_double * NJ), ("cmd", C.c_double * 3),
                ("air", C.c_double * 2), ("con", C.c_double * 2), ("tau", C.c_double * NJ), ("jacc", C.c_double * NJ),
                ("fmax_foot", C.c_double * 2), ("fmax_knee", C.c_double * 2), ("fmax_torso", C.c_double),
                ("eplen", C.c_int)]


class Report(C.Structure):
    _fields_ = [("foot_force", (C.c_double * 3) * 2), ("knee_force", (C.c_double * 3) * 2),
                ("torso_force", C.c_double * 3)]


_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        vp, dp = C.c_void_p, C.POINTER(C.c_double)
        M, Cf = C.POINTER(H12Model), C.POINTER(H12Config)
        L.orc_forward_dynamics.argtypes = [M, Cf, C.POINTER(Phys), dp, C.c_int, C.c_double, C.c_int, dp, C.POINTER(Report)]
        L.orc_mass_matrix.argtypes = [M, C.POINTER(Phys), dp]
        L.orc_energy_momentum.argtypes = [M, C.POINTER(Phys), dp, dp, dp]
        L.orc_self_contacts.argtypes = [M, Cf, C.POINTER(Phys), dp, C.POINTER(Report)]
        L.orc_body_poses.argtypes = [M, C.POINTER(Phys), dp, dp]
        L.orc_physics_step.argtypes = [M, Cf, C.POINTER(Phys), dp, C.c_int, C.c_int, C.POINTER(Report)]
        L.orc_mujoco_rollout.argtypes = [M, Cf, C.POINTER(Phys), dp, C.c_int, C.c_int, C.c_int, dp]
        L.orc_env_reset.argtypes = [M, Cf, C.c_int, C.c_int64, vp, vp, vp, vp, C.c_uint64]
        L.orc_env_step.argtypes = [M, Cf, C.c_int, C.c_int64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                   C.c_int64, C.c_int]
        L.orc_cat_reset.argtypes = []
        L.orc_cat_reset.restype = None
        L.orc_cat_running_max.argtypes = [dp]
        L.orc_cat_running_max.restype = None
        L.orc_cat_last_constraints.argtypes = [dp, C.c_int]
        L.orc_cat_last_constraints.restype = C.c_int
        L.orc_env_step_physics.argtypes = [M, Cf, C.c_int, vp, vp, vp, C.c_int]
        L.orc_env_observe.argtypes = [M, Cf, C.c_int, C.c_int64, vp, vp, vp, vp, vp, C.c_uint64]
        L.orc_delay_source.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_delay_source.restype = C.c_int
        L.orc_history_write.argtypes = [dp, vp, vp, C.c_int]
        L.orc_history_write.restype = None
        L.orc_philox.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]
        L.orc_philox.restype = None
        L.orc_set_terrain.argtypes = [vp, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, vp, C.c_int, C.c_int]
        L.orc_set_terrain.restype = None
        L.orc_ground.argtypes = [Cf, C.c_double, C.c_double, dp, dp]
        L.orc_ground.restype = C.c_double
        L.orc_obs_dim.argtypes = [Cf]
        L.orc_obs_dim.restype = C.c_int
        L.orc_set_dz_count.argtypes = [C.c_int]
        L.orc_set_dz_count.restype = None
        L.orc_dz_count.argtypes = []
        L.orc_dz_count.restype = C.c_int
        L.orc_set_self_jitter.argtypes = [C.c_double, C.c_uint64]
        L.orc_set_self_jitter.restype = None
        L.orc_set_threshold_jitter.argtypes = [C.c_double, C.c_double, C.c_uint64]
        L.orc_set_threshold_jitter.restype = None
        Tp = C.POINTER(TermIn)
        L.orc_mdp_terms.argtypes = [M, Cf, Tp, dp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.orc_mdp_terms.restype = C.c_int
        L.orc_cat_row.argtypes = [M, Cf, Tp, C.c_int, dp, dp, C.c_size_t]
        L.orc_cat_row.restype = C.c_int
        L.orc_cat_probs.argtypes = [Cf, C.c_int, dp, dp, C.POINTER(C.c_int), dp, dp, dp]
        L.orc_cat_probs.restype = C.c_int
        L.orc_cat_stats.argtypes = [Cf, C.c_int, dp, dp, vp, vp, vp, vp]
        L.orc_cat_stats.restype = None
        L.orc_cmd_update_decided.argtypes = [Cf, dp, C.c_double, dp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_cmd_update_decided.restype = C.c_int
        L.orc_terrain_move.argtypes = [Cf, dp, dp, dp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.orc_terrain_move.restype = None
        L.orc_obs_frame_from.argtypes = [Cf, dp, dp, dp]
        L.orc_obs_frame_from.restype = None
        L.orc_rough_row_from.argtypes = [Cf, dp, dp, vp]
        L.orc_rough_row_from.restype = None
        L.orc_history_write_n.argtypes = [dp, vp, vp, C.c_int, C.c_int]
        L.orc_history_write_n.restype = None
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _d(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def delay_source(lag, since_reset, substep, decimation):
    return lib().orc_delay_source(lag, since_reset, substep, decimation)


def history_write(frame, prev_row, fill):
    frame = np.ascontiguousarray(frame, dtype=np.float64)
    prev = np.ascontiguousarray(prev_row, dtype=np.float32)
    out = np.empty(NOBS, dtype=np.float32)
    lib().orc_history_write(_d(frame), _p(prev), _p(out), int(fill))
    return out


def term_in(state, act, act_prev, cmd, air, con, tau, jacc, fmax_foot, fmax_knee, fmax_torso, eplen) -> TermIn:
    """orc_term_in from numpy pieces; state = 37 physics coordinates (pos, quat wxyz, v_world, w_body, q, qd)."""
    t = TermIn()
    t.p = Phys.from_numpy(state)
    t.act[:] = np.asarray(act, np.float64)
    t.act_prev[:] = np.asarray(act_prev, np.float64)
    t.cmd[:] = np.asarray(cmd, np.float64)
    t.air[:] = np.asarray(air, np.float64)
    t.con[:] = np.asarray(con, np.float64)
    t.tau[:] = np.asarray(tau, np.float64)
    t.jacc[:] = np.asarray(jacc, np.float64)
    t.fmax_foot[:] = np.asarray(fmax_foot, np.float64)
    t.fmax_knee[:] = np.asarray(fmax_knee, np.float64)
    t.fmax_torso = float(fmax_torso)
    t.eplen = int(eplen)
    return t


def mdp_terms(model, cfg, ti: TermIn):
    """(20 unweighted reward terms, terminated, time_out) of one env snapshot."""
    out = np.zeros(20)
    term, tout = C.c_int(), C.c_int()
    lib().orc_mdp_terms(C.byref(model), C.byref(cfg), C.byref(ti), _d(out), C.byref(term), C.byref(tout))
    return out, bool(term.value), bool(tout.value)


def cat_row(model, cfg, ti: TermIn, terminated: bool, swing_h):
    """(58,) constraint values (+ still flag, episode length) of one env; swing_h (2,) updated in place."""
    out = np.zeros(58)
    sw = np.ascontiguousarray(swing_h, dtype=np.float64)
    lib().orc_cat_row(C.byref(model), C.byref(cfg), C.byref(ti), int(terminated), _d(sw), _d(out), 1)
    swing_h[:] = sw
    return out


class CaTProbs:
    """orc_cat_probs with its running maxima carried between calls (a fresh CaT object)."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.run_max = np.zeros(56)
        self.init = C.c_int(0)

    def __call__(self, cs):
        cs = np.ascontiguousarray(cs, dtype=np.float64)
        n = cs.shape[1]
        pmax, pterm, ceff = np.zeros(n), np.zeros((10, n)), np.zeros((56, n))
        lib().orc_cat_probs(C.byref(self.cfg), n, _d(cs), _d(self.run_max), C.byref(self.init), _d(pmax), _d(pterm),
                            _d(ceff))
        return pmax, pterm, ceff


def cat_stats(cfg, pterm, eplen, reset, sum_v, sum_p, log_acc):
    """orc_cat_stats on (10, n) episode sums (float32, updated in place) and a log accumulator (NLOG float32)."""
    pterm = np.ascontiguousarray(pterm, dtype=np.float64)
    eplen = np.ascontiguousarray(eplen, dtype=np.float64)
    reset = np.ascontiguousarray(reset, dtype=np.uint8)
    lib().orc_cat_stats(C.byref(cfg), pterm.shape[1], _d(pterm), _d(eplen), _p(reset), _p(sum_v), _p(sum_p),
                        _p(log_acc))


def cmd_update_decided(cfg, cmd, heading_target, quat, is_heading, is_standing, deactivate, activate, flip):
    c = np.ascontiguousarray(cmd, dtype=np.float64).copy()
    q = np.ascontiguousarray(quat, dtype=np.float64)
    r = lib().orc_cmd_update_decided(C.byref(cfg), _d(c), float(heading_target), _d(q), int(is_heading),
                                     int(is_standing), int(deactivate), int(activate), int(flip))
    return c, bool(r)


def terrain_move(cfg, pos, origin, cmd):
    up, down = C.c_int(), C.c_int()
    lib().orc_terrain_move(C.byref(cfg), _d(np.ascontiguousarray(pos, np.float64)),
                           _d(np.ascontiguousarray(origin, np.float64)), _d(np.ascontiguousarray(cmd, np.float64)),
                           C.byref(up), C.byref(down))
    return bool(up.value), bool(down.value)


def obs_frame_from(cfg, raw, u):
    raw = np.ascontiguousarray(raw, dtype=np.float64)
    u = np.ascontiguousarray(u, dtype=np.float64)
    fr = np.zeros(45)
    lib().orc_obs_frame_from(C.byref(cfg), _d(raw), _d(u), _d(fr))
    return fr


def rough_row_from(cfg, raw, u):
    raw = np.ascontiguousarray(raw, dtype=np.float64)
    u = np.ascontiguousarray(u, dtype=np.float64)
    out = np.zeros(235, dtype=np.float32)
    lib().orc_rough_row_from(C.byref(cfg), _d(raw), _d(u), _p(out))
    return out


def history_write_n(frame, prev_row, fill, nh):
    frame = np.ascontiguousarray(frame, dtype=np.float64)
    prev = np.ascontiguousarray(prev_row, dtype=np.float32)
    out = np.empty(45 * nh, dtype=np.float32)
    lib().orc_history_write_n(_d(frame), _p(prev), _p(out), int(fill), int(nh))
    return out


def philox(seed, c0, c1, c2, c3):
    out = (C.c_uint32 * 4)()
    lib().orc_philox(seed, c0, c1, c2, c3, out)
    return list(out)


def forward_dynamics(model, cfg, state, tau, algo=0, dt_impl=0.0, contact=True):
    s = Phys.from_numpy(state)
    tau = np.ascontiguousarray(tau, dtype=np.float64)
    nd = np.zeros(18)
    rep = Report()
    rc = lib().orc_forward_dynamics(C.byref(model), C.byref(cfg), C.byref(s), _d(tau), algo, dt_impl, int(contact),
                                    _d(nd), C.byref(rep))
    if rc:
        raise RuntimeError("oracle forward dynamics failed")
    return nd, rep


def mass_matrix(model, state):
    s = Phys.from_numpy(state)
    M = np.zeros((18, 18))
    lib().orc_mass_matrix(C.byref(model), C.byref(s), _d(M))
    return M


def self_contacts(model, cfg, state, mu=None):
    """Self-contact wrenches between the legs (body-coordinate spatial forces, (13, 6)) and the report.  mu: the
    env's randomised (static, dynamic) friction of the left and right sole (4 values; cfg.per_env_friction)."""
    s = Phys.from_numpy(state)
    if mu is not None:
        s.env_params = 1
        s.mu[:] = [float(x) for x in mu]
    f = np.zeros(13 * 6)
    rep = Report()
    lib().orc_self_contacts(C.byref(model), C.byref(cfg), C.byref(s), _d(f), C.byref(rep))
    return f.reshape(13, 6), rep


def body_poses(model, state):
    """World rotation (13, 3, 3) and origin (13, 3) of every body."""
    s = Phys.from_numpy(state)
    R = np.zeros(13 * 9)
    p = np.zeros(13 * 3)
    lib().orc_body_poses(C.byref(model), C.byref(s), _d(R), _d(p))
    return R.reshape(13, 3, 3), p.reshape(13, 3)


def energy_momentum(model, state):
    s = Phys.from_numpy(state)
    e = np.zeros(1)
    lin = np.zeros(3)
    ang = np.zeros(3)
    lib().orc_energy_momentum(C.byref(model), C.byref(s), _d(e), _d(lin), _d(ang))
    return float(e[0]), lin, ang


def physics_step(model, cfg, state, tau_pd, contact=True, algo=1):
    s = Phys.from_numpy(state)
    tau = np.ascontiguousarray(tau_pd, dtype=np.float64)
    rep = Report()
    if lib().orc_physics_step(C.byref(model), C.byref(cfg), C.byref(s), _d(tau), int(contact), algo, C.byref(rep)):
        raise RuntimeError("oracle physics step failed")
    return s.to_numpy(), rep


def mujoco_rollout(model, cfg, state, q_ref, n_steps, contact=False, algo=0):
    s = Phys.from_numpy(state)
    q_ref = np.ascontiguousarray(q_ref, dtype=np.float64)
    traj = np.zeros((n_steps, NJ))
    if lib().orc_mujoco_rollout(C.byref(model), C.byref(cfg), C.byref(s), _d(q_ref), n_steps, int(contact), algo,
                                _d(traj)):
        raise RuntimeError("oracle rollout failed")
    return s.to_numpy(), traj


_terrain_keepalive = None


def set_terrain(heights, hscale, x0, y0, origins=None):
    """Install the heightfield the oracle uses while cfg.terrain = 1 (process-global)."""
    global _terrain_keepalive
    h = np.ascontiguousarray(heights, dtype=np.float32)
    o = None if origins is None else np.ascontiguousarray(origins, dtype=np.float32)
    _terrain_keepalive = (h, o)
    rows, cols = (0, 0) if o is None else o.shape[:2]
    lib().orc_set_terrain(_p(h), h.shape[0], h.shape[1], float(hscale), float(x0), float(y0), _p(o), rows, cols)


def set_dz_count(v: int):
    """Deadzone command count the next step reads (the kernel's counter starts at 0)."""
    lib().orc_set_dz_count(int(v))


def cat_reset():
    """Forget the CaT running maxima (a fresh ConstraintManager)."""
    lib().orc_cat_reset()


def cat_running_max() -> np.ndarray:
    out = np.zeros(56)
    lib().orc_cat_running_max(_d(out))
    return out


def cat_last_constraints(n: int) -> np.ndarray:
    """(58, n): the last step's raw constraints (56 columns), no_move flag, pre-reset episode length."""
    out = np.zeros((58, n))
    if lib().orc_cat_last_constraints(_d(out), n):
        raise RuntimeError("no CaT step of that size")
    return out


def dz_count() -> int:
    return int(lib().orc_dz_count())


def set_self_jitter(eps: float, seed: int = 0):
    """Test hook: jitter every self-contact capsule end point by uniform +-eps m per coordinate (0 = exact)."""
    lib().orc_set_self_jitter(float(eps), int(seed) & 0xFFFFFFFFFFFFFFFF)


def set_threshold_jitter(lim_eps: float, contact_eps: float, seed: int = 0):
    """Test hook: decide every joint-limit / ground-contact switch with the limit (rad) / depth (m) shifted by a fresh
    uniform +-eps (0, 0 = exact; oracle/h12_oracle.c "test hooks")."""
    lib().orc_set_threshold_jitter(float(lim_eps), float(contact_eps), int(seed) & 0xFFFFFFFFFFFFFFFF)


def ground(cfg, x, y):
    gx, gy = np.zeros(1), np.zeros(1)
    h = lib().orc_ground(C.byref(cfg), float(x), float(y), _d(gx), _d(gy))
    return h, gx[0], gy[0]


class OracleEnv:
    """Batched oracle env on the same SoA workspace layout as libh12env."""

    def __init__(self, model, cfg, n, env_offset=0):
        self.model, self.cfg, self.n, self.env_offset = model, cfg, n, env_offset
        self.F = np.zeros((NF_FLOAT, n), dtype=np.float32)
        self.I = np.zeros((NF_INT, n), dtype=np.int32)
        self.obs = np.zeros((n, lib().orc_obs_dim(C.byref(cfg))), dtype=np.float32)
        self.reset_counter = 0
        self.observe_counter = 0

    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        lib().orc_env_reset(C.byref(self.model), C.byref(self.cfg), self.n, self.env_offset, _p(self.F), _p(self.I),
                            _p(m), _p(self.obs), self.reset_counter)
        self.reset_counter += 1
        return self.obs.copy()

    def step(self, actions, step_index, n_threads=1):
        a = np.ascontiguousarray(actions, dtype=np.float32)
        obs = np.empty_like(self.obs)
        rew = np.empty(self.n, dtype=np.float32)
        term = np.empty(self.n, dtype=np.uint8)
        trunc = np.empty(self.n, dtype=np.uint8)
        log = np.zeros(NLOG, dtype=np.float32)
        tq = np.empty((self.n, NJ), dtype=np.float32)
        ff = np.empty((self.n, 2), dtype=np.float32)
        cp = np.zeros(self.n, dtype=np.float32)
        rc = lib().orc_env_step(C.byref(self.model), C.byref(self.cfg), self.n, self.env_offset, _p(self.F), _p(self.I),
                                _p(a), _p(self.obs), _p(obs), _p(rew), _p(term), _p(trunc), _p(log), _p(tq), _p(ff),
                                _p(cp), step_index, n_threads)
        if rc:
            raise RuntimeError("oracle env step failed")
        self.obs = obs
        return obs.copy(), rew, term.astype(bool), trunc.astype(bool), dict(log=log, applied_torque=tq, foot_force=ff,
                                                                            cstr_prob=cp)

    def observe(self, fill_mask=None):
        m = None if fill_mask is None else np.ascontiguousarray(fill_mask, dtype=np.uint8)
        out = np.empty_like(self.obs)
        lib().orc_env_observe(C.byref(self.model), C.byref(self.cfg), self.n, self.env_offset, _p(self.F), _p(self.I),
                              _p(self.obs), _p(out), _p(m), self.observe_counter)
        self.observe_counter += 1
        self.obs = out
        return out.copy()

    def step_physics(self, q_ref, n_substeps):
        q = np.ascontiguousarray(q_ref, dtype=np.float32)
        if lib().orc_env_step_physics(C.byref(self.model), C.byref(self.cfg), self.n, _p(self.F), _p(self.I), _p(q),
                                      n_substeps):
            raise RuntimeError("oracle physics failed")
