"""`Isaac-Velocity-Flat-H12_12dof-v0` as a ManagerBasedRLEnv-compatible vectorised env on MI355X.

Mirrors the public surface of IsaacLab 2.1's ``ManagerBasedRLEnv`` that the reference's training
script reaches through ``RslRlVecEnvWrapper`` (scripts/rsl_rl/train.py:102,120; mirror of step()
in packages/biped_tasks/biped_tasks/utils/cat/cat_env.py:95-193):

  reset(seed=None, options=None) -> (obs_dict, extras)
  step(actions (N,12)) -> (obs_dict{"policy": (N,450)}, rew (N,), terminated (N,), truncated (N,), extras)
  num_envs, device, step_dt, physics_dt, max_episode_length(_s), episode_length_buf (writable),
  cfg, observation_manager.group_obs_dim, action_manager.total_action_dim, unwrapped, close()

Every step is ONE launch of the fused HIP kernel in libh12env.so (no CPU fallback: a missing
extension raises).  State lives in one device workspace owned by a torch uint8 tensor; fields are
exposed as zero-copy torch views.
"""
from __future__ import annotations

import ctypes as C
import math
import weakref
from types import SimpleNamespace

import torch

from . import _abi
from ._abi import F as FIELDS
from ._abi import LOG_METRIC, NCSTR, NF_FLOAT, NF_INT, NJ, NLOG, NOBS_ROUGH, NREW, H12StepOut, check, load_library
from .cfg import H12FlatEnvCfg
from .model import body_names, build_model, joint_names

_LOG_RING = 128   # log accumulator slots (zeroed in chunks, see _log_slot)
_LOG_CHUNK = 32
_LOG_LOOKBACK = _LOG_RING - 2 * _LOG_CHUNK  # persistence of extras["log"] (see _LazyLog)


def env_origins_grid(num_envs: int, spacing: float, device) -> torch.Tensor:
    """TerrainImporter._compute_env_origins_grid (plane terrain): row/col grid centred at 0."""
    num_rows = math.ceil(num_envs / int(math.sqrt(num_envs)))
    num_cols = math.ceil(num_envs / num_rows)
    ii, jj = torch.meshgrid(torch.arange(num_rows, device=device), torch.arange(num_cols, device=device), indexing="ij")
    origins = torch.zeros(num_envs, 3, device=device)
    origins[:, 0] = -(ii.flatten()[:num_envs] - (num_rows - 1) / 2) * spacing
    origins[:, 1] = (jj.flatten()[:num_envs] - (num_cols - 1) / 2) * spacing
    return origins


def _raw_stream(dev_index: int) -> int:
    """The current HIP stream of the device as a raw pointer (what torch.cuda.current_stream().cuda_stream
    returns, without building a Stream object on every step)."""
    return torch._C._cuda_getCurrentRawStream(dev_index)


class _LazyLog(dict):
    """extras["log"]: IsaacLab's Episode_Reward/*, Episode_Termination/* and Metrics/base_velocity/* values,
    materialised on first access from the step's device-side accumulator (no host sync inside step()).

    Persistence (cat_env.py:217-245 / ManagerBasedRLEnv.step): the reference rebuilds extras["log"] only in
    _reset_idx, i.e. on steps where some env resets; on a step without resets extras["log"] still holds the last
    such step's values.  On materialisation the log therefore reads the most recent accumulator slot, this
    step's or an earlier one within _LOG_LOOKBACK steps, that counts a reset (device-side gather, no host sync;
    nothing is kept alive or computed per step for logs nobody reads)."""

    def __init__(self, ring: torch.Tensor, slot: int, max_episode_length_s: float, terms: list, term_map: torch.Tensor,
                 cstr: list | None = None, extra: dict | None = None, lookback: int = 1, flush=None):
        super().__init__()
        self._flush = flush  # completes the library's deferred accumulator additions (h12env_flush_log)
        self._ring = ring
        self._slot = slot
        self._lookback = lookback
        self._T = max_episode_length_s
        self._terms = terms          # [(cfg name, kernel ids)] in RewardManager order
        self._map = term_map         # (terms, NREW) 0/1: a cfg term sums its kernel ids
        self._cstr = cstr or []      # [(constraint name, kernel constraint id)]
        self._extra = extra or {}
        self._keys = None  # built on first access (step() stays cheap for logs nobody reads)
        self._done = False

    def _key_list(self):
        if self._keys is None:
            keys = [f"Episode_Reward/{t}" for t, _ in self._terms]
            keys += [f"Episode_Constraint_violation/{c}" for c, _ in self._cstr]
            keys += [f"Episode_Constraint_probability/{c}" for c, _ in self._cstr]
            keys += ["Metrics/base_velocity/error_vel_xy", "Metrics/base_velocity/error_vel_yaw",
                     "Episode_Termination/time_out", "Episode_Termination/base_contact"]
            self._nt = len(keys)
            self._keys = keys + list(self._extra)
        return self._keys

    def _fill(self):
        if self._done:
            return
        if self._flush is not None:
            self._flush()
        ring = self._ring
        idx = (self._slot - torch.arange(self._lookback, device=ring.device)) % ring.shape[0]
        k = torch.argmax((ring[idx, NREW] > 0).to(torch.int32)).view(1)  # first slot counting a reset (0 if none)
        a = ring.index_select(0, idx.index_select(0, k))[0]  # device-side gather (a tensor index would sync)
        n = a[NREW].clamp(min=1.0)
        parts = [self._map @ a[:NREW] / n / self._T]
        if self._cstr:
            cid = torch.tensor([k for _, k in self._cstr], device=a.device, dtype=torch.long)
            parts += [a[NREW + 4 + cid] / n * 100.0, a[NREW + 4 + NCSTR + cid] / n]
        parts += [a[LOG_METRIC:LOG_METRIC + 2] / n, a[NREW + 1:NREW + 3]]
        vals = torch.cat(parts)
        keys = self._key_list()
        for i, k in enumerate(keys[:self._nt]):
            dict.__setitem__(self, k, vals[i])
        for k, f in self._extra.items():
            dict.__setitem__(self, k, f())
        self._done = True

    def __getitem__(self, k):
        self._fill()
        return dict.__getitem__(self, k)

    def keys(self):
        self._fill()
        return dict.keys(self)

    def items(self):
        self._fill()
        return dict.items(self)

    def values(self):
        self._fill()
        return dict.values(self)

    def __iter__(self):
        self._fill()
        return dict.__iter__(self)

    def __len__(self):
        return len(self._key_list())

    def __contains__(self, k):
        return k in self._key_list()


class _ObservationManager:
    def __init__(self, env):
        self._env = env
        self.group_obs_dim = {"policy": (env.obs_dim,)}
        self.group_obs_concatenate = {"policy": True}
        terms = ["base_ang_vel", "projected_gravity", "velocity_commands", "joint_pos", "joint_vel", "actions"]
        if env.obs_dim == NOBS_ROUGH:
            terms = ["base_lin_vel"] + terms + ["height_scan"]
        self.active_terms = {"policy": terms}

    def compute(self):
        return {"policy": self._env._obs[self._env._k]}


class _RewardManager:
    """RewardManager surface used by curriculum terms (modify_reward_weight): term names in order and
    get/set_term_cfg; a weight change is pushed to the kernel (h12env_set_reward_weights)."""

    def __init__(self, env):
        self._env = env

    @property
    def active_terms(self):
        return [k for k, _ in self._env.cfg.rewards.active()]

    def get_term_cfg(self, name):
        t = dict(self._env.cfg.rewards.items()).get(name)
        if t is None:
            raise ValueError(f"reward term {name!r} not found")
        return t

    def set_term_cfg(self, name, term_cfg):
        setattr(self._env.cfg.rewards, name, term_cfg)
        self._env._push_reward_weights()


class _ConstraintManager:
    """ConstraintManager surface (T/utils/cat/constraint_manager.py:126-269) over the kernel's constraint terms:
    active terms in order, get/set_term_cfg (max_p reaches the kernel via h12env_set_constraint_max_p)."""

    def __init__(self, env):
        self._env = env

    @property
    def active_terms(self):
        return [k for k, _ in self._env.cfg.constraints.active()]

    def get_term_cfg(self, name):
        t = dict(self._env.cfg.constraints.items()).get(name)
        if t is None:
            raise ValueError(f"Constraint term '{name}' not found.")
        return t

    def set_term_cfg(self, name, term_cfg):
        if name not in self.active_terms:
            raise ValueError(f"Constraint term '{name}' not found.")
        setattr(self._env.cfg.constraints, name, term_cfg)
        self._env._push_constraint_p()


class _ActionManager:
    def __init__(self, env):
        self._env = env
        self.total_action_dim = NJ
        self.action_term_dim = [NJ]

    @property
    def action(self):
        return self._env._field("ACT").T

    @property
    def prev_action(self):
        return self._env._field("ACT_PREV").T


class _ArticulationData:
    """Zero-copy (N, k) views of the SoA workspace in IsaacLab's ArticulationData vocabulary."""

    def __init__(self, env):
        self._env = env
        self.joint_names = joint_names()
        self.body_names = body_names()
        dev = env.device
        m = build_model()
        self.default_joint_pos = torch.tensor(list(m.q_default), device=dev).repeat(env.num_envs, 1)
        self.default_joint_vel = torch.zeros(env.num_envs, NJ, device=dev)
        lo = torch.tensor(list(m.q_lower), device=dev)
        hi = torch.tensor(list(m.q_upper), device=dev)
        self.joint_pos_limits = torch.stack([lo, hi], -1).repeat(env.num_envs, 1, 1)
        f = env.cfg.robot.soft_joint_pos_limit_factor
        mid, half = (lo + hi) / 2, (hi - lo) / 2 * f
        self.soft_joint_pos_limits = torch.stack([mid - half, mid + half], -1).repeat(env.num_envs, 1, 1)

    @property
    def joint_pos(self):
        return self._env._field("Q").T

    @property
    def joint_vel(self):
        return self._env._field("QD").T

    @property
    def root_pos_w(self):
        e = self._env
        # terrain tasks keep world positions in the workspace; the plane keeps env-local ones
        return e._field("POS").T if e.terrain is not None else e._field("POS").T + e.scene.env_origins

    @property
    def root_quat_w(self):
        return self._env._field("QUAT").T

    @property
    def root_ang_vel_b(self):
        return self._env._field("WANG").T

    @property
    def root_link_lin_vel_w(self):
        return self._env._field("VLIN").T


class H12VelocityEnv:
    """Drop-in for ``ManagerBasedRLEnv`` on ``Isaac-Velocity-Flat-H12_12dof-v0``."""

    is_vector_env = True
    metadata = {"render_modes": [None], "isaac_sim_version": "none (MI355X-native)"}

    def __init__(self, cfg: H12FlatEnvCfg | None = None, render_mode: str | None = None, env_offset: int = 0,
                 obs_copy: bool = False, **kwargs):
        self.cfg = cfg if cfg is not None else H12FlatEnvCfg()
        self.render_mode = render_mode
        self.device = torch.device(self.cfg.sim.device)
        if self.device.type != "cuda":
            raise RuntimeError(f"H12VelocityEnv runs on the MI355X HIP path only (device={self.device})")
        self.num_envs = int(self.cfg.scene.num_envs)
        self.env_offset = int(env_offset)
        self.obs_copy = obs_copy
        self._lib = load_library()
        self._model = build_model()
        self._ccfg = self.cfg.to_c()
        torch.cuda.set_device(self.device)
        nbytes = self._lib.h12env_state_bytes(self.num_envs)
        self._state = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)
        h = C.c_void_p()
        check(self._lib, self._lib.h12env_create(C.byref(self._model), C.byref(self._ccfg), self.num_envs,
                                                 self.env_offset, self.device.index or 0,
                                                 C.c_void_p(self._state.data_ptr()), C.byref(h)), "h12env_create")
        self._h = h
        self._fstate = self._state.view(torch.float32)[: NF_FLOAT * self.num_envs].view(NF_FLOAT, self.num_envs)
        self._istate = self._state.view(torch.int32)[NF_FLOAT * self.num_envs:].view(NF_INT, self.num_envs)
        n = self.num_envs
        self.obs_dim = int(self._lib.h12env_obs_dim(h))
        self._obs = [torch.zeros(n, self.obs_dim, device=self.device), torch.zeros(n, self.obs_dim, device=self.device)]
        self._k = 0
        self.reward_buf = torch.zeros(n, device=self.device)
        self.reset_terminated = torch.zeros(n, dtype=torch.bool, device=self.device)
        self.reset_time_outs = torch.zeros(n, dtype=torch.bool, device=self.device)
        self.reset_buf = self.reset_terminated
        self._log_ring = torch.zeros(_LOG_RING, NLOG, device=self.device)
        self._live_logs: dict = {}  # creation step -> weakref of the _LazyLog reading the ring
        self._applied_torque = torch.zeros(n, NJ, device=self.device)
        # |net contact force| of the left / right foot over the last physics step (ContactSensor of the feet)
        self.foot_contact_force = torch.zeros(n, 2, device=self.device)
        self._step_outs = []  # per observation buffer: (H12StepOut, byref), see _build_step_outs
        self._rollout = None  # bind_rollout: compact rollout records written by the step kernels
        self.common_step_counter = 0
        self.extras: dict = {}
        self.terrain = None
        self._apply_startup()
        if self.terrain is not None:
            origins = self._field("ORIGIN").T  # moved in-kernel by the terrain curriculum
        else:
            origins = env_origins_grid(n, self.cfg.scene.env_spacing, self.device)
        self.scene = SimpleNamespace(env_origins=origins, num_envs=n, terrain=self.terrain)
        self.observation_manager = _ObservationManager(self)
        self.action_manager = _ActionManager(self)
        self.reward_manager = _RewardManager(self)
        self._set_reward_terms()
        self._rw_pending = list(getattr(self.cfg.curriculum, "reward_weights", []) or [])
        # CaT (Isaac-Velocity-CaT-Flat-H12_12dof-v0): constraint probabilities -> dones
        self._cat = self.cfg.constraints is not None
        self._cstr_terms = self.cfg.constraints.active() if self._cat else []
        self._cp_terms = list(getattr(self.cfg.curriculum, "constraint_p", []) or []) if self._cat else []
        self._cstr_p_pushed = None
        self._cstr_p_buf = (C.c_float * NCSTR)()
        if self._cat:
            self.constraint_manager = _ConstraintManager(self)
            self._dones = torch.zeros(n, device=self.device)
        self._build_step_outs()
        self._data = _ArticulationData(self)
        self.scene.articulations = {"robot": SimpleNamespace(data=self._data, joint_names=self._data.joint_names,
                                                             body_names=self._data.body_names,
                                                             num_joints=NJ)}
        self.scene.__dict__["robot"] = self.scene.articulations["robot"]
        self._configure_spaces()
        self._closed = False

    def _build_step_outs(self):
        """h12env_step output structs, one per observation buffer (their pointers never change), the log ring's
        base pointer and the log's extra terms: step() then only sets the log slot."""
        self._dev_index = self.device.index or 0
        self._act_shape = torch.Size((self.num_envs, NJ))
        self._step_outs = []
        for k in range(2):
            o = H12StepOut()
            o.obs = self._obs[k].data_ptr()
            o.rew = self.reward_buf.data_ptr()
            o.terminated = self.reset_terminated.data_ptr()
            o.truncated = self.reset_time_outs.data_ptr()
            o.applied_torque = self._applied_torque.data_ptr()
            o.foot_force = self.foot_contact_force.data_ptr()
            o.cstr_prob = self._dones.data_ptr() if self._cat else None
            self._step_outs.append((o, C.byref(o)))
        self._log_ptr = self._log_ring.data_ptr()
        self._log_extra = ({"Curriculum/terrain_levels": lambda: self.terrain_levels().mean()}
                           if self.terrain is not None else None)

    # ------------------------------------------------------------------ properties (ManagerBasedEnv)
    @property
    def unwrapped(self):
        return self

    @property
    def physics_dt(self) -> float:
        return self.cfg.sim.dt

    @property
    def step_dt(self) -> float:
        return self.cfg.sim.dt * self.cfg.decimation

    @property
    def max_episode_length_s(self) -> float:
        return self.cfg.episode_length_s

    @property
    def max_episode_length(self) -> int:
        return math.ceil(self.max_episode_length_s / self.step_dt)

    @property
    def episode_length_buf(self) -> torch.Tensor:
        return self._istate[_abi.I["EPLEN"][0]]

    @episode_length_buf.setter
    def episode_length_buf(self, value: torch.Tensor):
        self._istate[_abi.I["EPLEN"][0]].copy_(value.to(self.device))

    @property
    def obs_buf(self):
        return {"policy": self._obs[self._k]}

    def _field(self, name: str) -> torch.Tensor:
        off, cnt = FIELDS[name]
        return self._fstate[off:off + cnt]

    def _configure_spaces(self):
        try:
            import gymnasium as gym
            import numpy as np

            self.single_observation_space = gym.spaces.Dict(
                {"policy": gym.spaces.Box(low=-np.inf, high=np.inf, shape=(self.obs_dim,))})
            self.single_action_space = gym.spaces.Box(low=-np.inf, high=np.inf, shape=(NJ,))
            self.observation_space = gym.vector.utils.batch_space(self.single_observation_space, self.num_envs)
            self.action_space = gym.vector.utils.batch_space(self.single_action_space, self.num_envs)
        except Exception:  # gymnasium is optional for the hot path
            self.single_observation_space = {"policy": (self.obs_dim,)}
            self.single_action_space = (NJ,)
            self.observation_space = {"policy": (self.num_envs, self.obs_dim)}
            self.action_space = (self.num_envs, NJ)

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------ rough task: terrain + startup events
    def _apply_startup(self):
        """Terrain (TerrainGenerator + TerrainImporter curriculum origins) and mode="startup" events,
        computed on the host by h12env.startup and written into the workspace once."""
        from .startup import startup_state

        st = startup_state(self.cfg, self.num_envs, self.env_offset)
        self.terrain = st.terrain
        for name, val in st.fields.items():
            self._field(name).copy_(torch.from_numpy(val).to(self.device))
        if st.terrain_cell is not None:
            self._istate[_abi.I["TERRAIN"][0]].copy_(torch.from_numpy(st.terrain_cell).to(self.device))
        if self.terrain is not None:
            self._t_heights = torch.from_numpy(self.terrain.heights).to(self.device)
            self._t_origins = torch.from_numpy(self.terrain.origins).to(self.device)
            self._bind_terrain()

    def _bind_terrain(self):
        t = self.terrain
        if t is None:
            return
        rows, cols = t.origins.shape[:2]
        check(self._lib, self._lib.h12env_set_terrain(self._h, C.c_void_p(self._t_heights.data_ptr()), t.shape[0],
                                                       t.shape[1], t.hscale, t.x0, t.y0,
                                                       C.c_void_p(self._t_origins.data_ptr()), rows, cols),
              "h12env_set_terrain")

    def _set_reward_terms(self):
        self._reward_terms = self.cfg.rewards.active()
        m = torch.zeros(len(self._reward_terms), NREW, device=self.device)
        for i, (_, ids) in enumerate(self._reward_terms):
            m[i, list(ids)] = 1.0
        self._reward_map = m

    def _push_constraint_p(self):
        """max_p of the active constraint terms -> the kernel, only when a value changed (no config rebuild)."""
        terms = dict(self.cfg.constraints.items())
        vals = list(self._cstr_p_pushed) if self._cstr_p_pushed is not None else list(self._ccfg.cstr_max_p)
        for name, cid in self._cstr_terms:
            vals[cid] = float(terms[name].max_p)
        if vals == self._cstr_p_pushed:
            return
        self._cstr_p_buf[:] = vals
        check(self._lib, self._lib.h12env_set_constraint_max_p(self._h, self._cstr_p_buf, NCSTR),
              "h12env_set_constraint_max_p")
        self._cstr_p_pushed = vals

    def _constraint_curriculum(self):
        """modify_constraint_p runs in _reset_idx after the constraints of a step: step t uses the max_p
        computed with common_step_counter t - 1 (the first step: the initial reset's counter 0)."""
        for t in self._cp_terms:
            self.constraint_manager.get_term_cfg(t.term_name).max_p = t.max_p(self.common_step_counter - 1)
        self._push_constraint_p()

    def _push_reward_weights(self):
        self._ccfg = self.cfg.to_c()
        self._set_reward_terms()
        w = (C.c_float * NREW)(*self._ccfg.rew_w)
        check(self._lib, self._lib.h12env_set_reward_weights(self._h, w, NREW), "h12env_set_reward_weights")

    def _reward_curriculum(self):
        """modify_reward_weight terms: CurriculumManager.compute runs in _reset_idx after the rewards of a
        step, so a term whose num_steps the previous step passed reweights from this step on."""
        due = [t for t in self._rw_pending if self.common_step_counter - 1 > t.num_steps]
        if not due:
            return
        for t in due:
            term = self.reward_manager.get_term_cfg(t.term_name)
            term.weight = t.weight
            self._rw_pending.remove(t)
        self._push_reward_weights()

    def terrain_levels(self) -> torch.Tensor:
        return (self._istate[_abi.I["TERRAIN"][0]] & 0xFFFF).float()

    # ------------------------------------------------------------------ gym API
    def seed(self, seed: int = -1) -> int:
        self.cfg.seed = int(seed)
        self._ccfg = self.cfg.to_c()
        # rebuild the kernel parameters with the new seed, keeping the workspace
        h = C.c_void_p()
        check(self._lib, self._lib.h12env_create(C.byref(self._model), C.byref(self._ccfg), self.num_envs,
                                                 self.env_offset, self.device.index or 0,
                                                 C.c_void_p(self._state.data_ptr()), C.byref(h)), "h12env_create")
        self._lib.h12env_destroy(self._h)
        self._h = h
        self._bind_terrain()
        return int(seed)

    def reset(self, seed: int | None = None, env_ids=None, options=None):
        self._no_bound_rollout("reset()")
        if seed is not None:
            self.seed(seed)
        mask = None
        if env_ids is not None:
            mask = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
            mask[torch.as_tensor(env_ids, device=self.device, dtype=torch.long)] = 1
        obs = self._obs[self._k]
        check(self._lib, self._lib.h12env_reset(self._h, None if mask is None else C.c_void_p(mask.data_ptr()),
                                                C.c_void_p(obs.data_ptr()), self._stream()), "h12env_reset")
        self.extras = {}
        return {"policy": obs.clone() if self.obs_copy else obs}, self.extras

    def step(self, action: torch.Tensor):
        a = action
        if a.device != self.device or a.dtype != torch.float32 or not a.is_contiguous():
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
        if a.shape != self._act_shape:
            raise ValueError(f"actions must be ({self.num_envs}, {NJ}), got {tuple(a.shape)}")
        self.common_step_counter += 1
        if self._rw_pending:
            self._reward_curriculum()
        if self._cp_terms:
            self._constraint_curriculum()
        prev = self._obs[self._k]
        self._k ^= 1
        obs = self._obs[self._k]
        slot = self.common_step_counter % _LOG_RING
        if slot % _LOG_CHUNK == 0:
            # a step's _LazyLog reads the ring lazily (its slot, or up to _LOG_LOOKBACK - 1 earlier ones): the
            # chunk recycled now held steps C - RING .. C - RING + CHUNK - 1, so every log still alive whose window
            # reaches into it (created at step <= C - RING + CHUNK + LOOKBACK - 2) is materialised first (device
            # ops, no sync); newer logs, e.g. the one extras still holds, are left lazy
            c = self.common_step_counter
            for t0 in list(self._live_logs):
                log = self._live_logs[t0]()
                if log is None:
                    del self._live_logs[t0]
                elif t0 <= c - _LOG_RING + _LOG_CHUNK + _LOG_LOOKBACK - 2:
                    log._fill()
                    del self._live_logs[t0]
            self._flush_log()  # no deferred fold may land in the recycled slots after the zeroing
            self._log_ring[slot:slot + _LOG_CHUNK].zero_()
        # the output pointers are fixed per observation buffer (built once, _step_outs); only the log slot moves
        rec = self._rollout
        if rec is None:
            o, o_ref = self._step_outs[self._k]
        else:  # rollout record t: reward, done flags and the new frame go straight into it
            t = rec.t
            o, o_ref = self._rollout_outs[self._k]
            o.rew, o.terminated, o.truncated, o.frame_out = self._rollout_ptrs[t]
            self.reward_buf, self.reset_terminated, self.reset_time_outs = self._rollout_views[t]
            self.reset_buf = self.reset_terminated
            rec.t = t + 1 if t + 1 < rec.slots else 0
        o.log_acc = self._log_ptr + slot * (NLOG * 4)
        rc = self._lib.h12env_step(self._h, a.data_ptr(), prev.data_ptr(), o_ref, self.common_step_counter,
                                   _raw_stream(self._dev_index))
        if rc:
            check(self._lib, rc, "h12env_step")
        log = _LazyLog(self._log_ring, slot, self.max_episode_length_s, self._reward_terms, self._reward_map,
                       self._cstr_terms, self._log_extra, _LOG_LOOKBACK, self._flush_and_check)
        self._live_logs[self.common_step_counter] = weakref.ref(log)
        self.extras = {"log": log, "time_outs": self.reset_time_outs}
        obs_out = obs.clone() if self.obs_copy else obs
        if self._cat:  # CaTEnv.step: dones = constraint termination probability, 1 where reset (cat_env.py:153-193)
            return {"policy": obs_out}, self.reward_buf, self._dones, self.reset_time_outs, self.extras
        return {"policy": obs_out}, self.reward_buf, self.reset_terminated, self.reset_time_outs, self.extras

    def bind_rollout(self, rec):
        """Record every following step into the compact rollout ``rec`` (h12env.rollout.RolloutRecorder; BASELINE
        config C4): the step's reward, terminated / truncated flags and new observation frame (as it enters the
        history) are written by the kernels straight into ring slot ``rec.t``, which then advances (mod rec.slots); the
        returned reward / flag tensors are views of that record.  Flat observation layout only (the frames rebuild
        the history rows).  Only step() may run while it is bound: reset() / observe() raise (their rows would not be in
        the records) -- unbind, reset, and bind a fresh recorder."""
        if self.obs_dim == NOBS_ROUGH or self._cat:
            raise ValueError("bind_rollout needs the flat observation layout (history) and a non-CaT task")
        if rec.n != self.num_envs or rec.history * 45 != self.obs_dim:
            raise ValueError("rollout recorder was built for another env shape")
        self._rollout_saved = (self.reward_buf, self.reset_terminated, self.reset_time_outs)
        self._rollout_ptrs = [(rec.rewards[t].data_ptr(), rec.terminated[t].data_ptr(), rec.truncated[t].data_ptr(),
                               rec.frames[t].data_ptr()) for t in range(rec.slots)]
        self._rollout_views = [(rec.rewards[t], rec.terminated[t], rec.truncated[t]) for t in range(rec.slots)]
        self._rollout_outs = []
        for k in range(2):
            o = H12StepOut()
            src = self._step_outs[k][0]
            for name, _ in H12StepOut._fields_:
                setattr(o, name, getattr(src, name))
            self._rollout_outs.append((o, C.byref(o)))
        self._rollout = rec

    def _no_bound_rollout(self, what):
        # only step() writes rollout records: a reset / observe in the middle of a recorded rollout would change the
        # history rows without a frame or done flag in the records, and h12env_rollout_decode would rebuild rows
        # that differ from the ones the env returned
        if getattr(self, "_rollout", None) is not None:
            raise RuntimeError(f"{what} while a rollout recorder is bound: call unbind_rollout() first")

    def unbind_rollout(self):
        if self._rollout is not None:
            self.reward_buf, self.reset_terminated, self.reset_time_outs = self._rollout_saved
            self.reset_buf = self.reset_terminated
            self._rollout = None

    def step_physics(self, q_ref: torch.Tensor, n_substeps: int):
        """Parity hook: physics only, PD towards a held joint target (h12env_step_physics)."""
        q = q_ref.to(device=self.device, dtype=torch.float32).contiguous()
        check(self._lib, self._lib.h12env_step_physics(self._h, C.c_void_p(q.data_ptr()), int(n_substeps),
                                                       self._stream()), "h12env_step_physics")

    def eval_terms(self, tau: torch.Tensor, jacc: torch.Tensor, fmax: torch.Tensor):
        """Parity hook (h12env_eval_terms): step()'s reward-term / termination / CaT-constraint code on the
        workspace state as it stands, with injected applied torques (N, 12), joint accelerations (N, 12) and
        per-body contact-history maxima (N, 5: feet L/R, knees L/R, torso).  Returns (terms (NREW, N),
        terminated (N,) bool, truncated (N,) bool, constraint rows (NCSTR_COLS + 4, N) or None: the raw columns,
        no_move flag, pre-reset episode length, and foot_clearance's updated swing height (left, right) -- the hook
        itself leaves the workspace unchanged)."""
        n = self.num_envs
        f = lambda x, k: x.to(device=self.device, dtype=torch.float32).contiguous().reshape(n, k)  # noqa: E731
        tau, jacc, fmax = f(tau, NJ), f(jacc, NJ), f(fmax, 5)
        terms = torch.zeros(NREW, n, device=self.device)
        term = torch.zeros(n, dtype=torch.uint8, device=self.device)
        trunc = torch.zeros(n, dtype=torch.uint8, device=self.device)
        cstr = torch.zeros(_abi.NCSTR_COLS + 4, n, device=self.device) if self._cat else None
        check(self._lib, self._lib.h12env_eval_terms(
            self._h, C.c_void_p(tau.data_ptr()), C.c_void_p(jacc.data_ptr()), C.c_void_p(fmax.data_ptr()),
            C.c_void_p(terms.data_ptr()), C.c_void_p(term.data_ptr()), C.c_void_p(trunc.data_ptr()),
            None if cstr is None else C.c_void_p(cstr.data_ptr()), self._stream()), "h12env_eval_terms")
        return terms, term.bool(), trunc.bool(), cstr

    def eval_self_contacts(self) -> torch.Tensor:
        """Parity hook (h12env_eval_self_contacts): the self-contact wrenches between the legs on the workspace
        state as it stands, (N, 2 legs, 2 bodies [knee, foot], 6 [moment, force]) in body coordinates."""
        out = torch.zeros(self.num_envs, 2, 2, 6, device=self.device)
        check(self._lib, self._lib.h12env_eval_self_contacts(self._h, C.c_void_p(out.data_ptr()), self._stream()),
              "h12env_eval_self_contacts")
        return out

    def observe(self, fill_mask: torch.Tensor | None = None):
        """ObservationManager.compute(): append a frame of the current state to the history."""
        self._no_bound_rollout("observe()")
        prev = self._obs[self._k]
        self._k ^= 1
        out = self._obs[self._k]
        fm = None if fill_mask is None else fill_mask.to(device=self.device, dtype=torch.uint8).contiguous()
        check(self._lib, self._lib.h12env_observe(self._h, C.c_void_p(prev.data_ptr()), C.c_void_p(out.data_ptr()),
                                                  None if fm is None else C.c_void_p(fm.data_ptr()),
                                                  self._stream()), "h12env_observe")
        return {"policy": out}

    def get_observations(self):
        return {"policy": self._obs[self._k]}

    def snapshot(self) -> dict:
        """Device copy of everything step() reads (workspace, both observation buffers, step counter), so a
        window of steps can be replayed bit for bit with restore().  The library-internal carries of the
        deadzone command count and the CaT running maxima are not included (Flat / Rough tasks only)."""
        return {"state": self._state.clone(), "obs": [o.clone() for o in self._obs], "k": self._k,
                "counter": self.common_step_counter}

    def restore(self, snap: dict):
        self._flush_log()  # folds of steps before the restore land in their own slots first
        self._state.copy_(snap["state"])
        for o, s in zip(self._obs, snap["obs"]):
            o.copy_(s)
        self._k = snap["k"]
        self.common_step_counter = snap["counter"]

    def render(self, recompute: bool = False):
        return None

    def _flush_log(self):
        if not self._closed:
            check(self._lib, self._lib.h12env_flush_log(self._h, _raw_stream(self._dev_index)), "h12env_flush_log")

    def check_device(self):
        """Synchronise and read the library's device diagnostic word (h12env_check): raises H12EnvError when a
        self-contact wait in the step kernel ended at its bound since the last check (that inner step's self-contact
        wrenches may be partial; H12EnvError is a RuntimeError).  Called where the host synchronises anyway:
        episode-log reads and close()."""
        if not self._closed and hasattr(self._lib, "h12env_check"):
            check(self._lib, self._lib.h12env_check(self._h, _raw_stream(self._dev_index)), "h12env_check")

    def _flush_and_check(self):
        self._flush_log()
        self.check_device()

    def close(self):
        if not self._closed:
            self._flush_log()  # logs still referenced (extras) stay complete
            torch.cuda.synchronize(self.device)
            rc = self._lib.h12env_check(self._h, _raw_stream(self._dev_index)) if hasattr(self._lib, "h12env_check") else 0
            msg = self._lib.h12env_last_error().decode() if rc else ""
            self._lib.h12env_destroy(self._h)
            self._closed = True
            if rc:
                raise _abi.H12EnvError(f"h12env_check failed ({rc}): {msg}")

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ accounting
    def step_cost(self):
        b, f = C.c_double(), C.c_double()
        self._lib.h12env_step_cost(self._h, C.byref(b), C.byref(f))
        return b.value, f.value

    @property
    def obs_fused(self) -> bool:
        """step() assembles the observation rows inside the env kernel (h12env_obs_fused); kernel 1 of the timing /
        cost pairs is then the deferred episode-log fold, else the observation assembly kernel."""
        return bool(self._lib.h12env_obs_fused(self._h))

    @property
    def cat_inline(self) -> bool:
        """CaT: step() applies the constraint probabilities inside the env kernel (h12env_cat_inline), with no
        separate probability kernel after it."""
        return hasattr(self._lib, "h12env_cat_inline") and bool(self._lib.h12env_cat_inline(self._h))

    def kernel_cost(self, kernel: int):
        """(compulsory HBM bytes, counted FLOPs) per env of kernel 0 (env step) or 1 (obs assembly, or the log fold
        per step on the fused path)."""
        b, f = C.c_double(), C.c_double()
        check(self._lib, self._lib.h12env_kernel_cost(self._h, kernel, C.byref(b), C.byref(f)), "h12env_kernel_cost")
        return b.value, f.value

    def set_kernel_timing(self, enable: bool):
        """Instrumentation: record HIP events around the two kernels of every step (off by default)."""
        check(self._lib, self._lib.h12env_set_kernel_timing(self._h, int(enable)), "h12env_set_kernel_timing")

    def kernel_times(self):
        """(env-kernel ms, obs-kernel ms, timed steps) summed since timing was enabled / last read."""
        a, b, n = C.c_double(), C.c_double(), C.c_int()
        check(self._lib, self._lib.h12env_kernel_times(self._h, C.byref(a), C.byref(b), C.byref(n)), "h12env_kernel_times")
        return a.value, b.value, n.value
