"""CPU toy env with the ManagerBasedRLEnv surface the rsl_rl wrapper and runner use (test double for the
PPO / shim tests; the H1-2 env itself needs the MI355X).  Task: drive a 3-D point to a per-env target;
obs = (target - x, x), reward = -|target - x|^2, episodes of 50 steps, random time-outs."""
from __future__ import annotations

from dataclasses import dataclass, field
from types import SimpleNamespace

import torch


@dataclass
class ToySceneCfg:
    num_envs: int = 64


@dataclass
class ToySimCfg:
    device: str = "cpu"


@dataclass
class ToyEnvCfg:
    seed: int | None = 0
    scene: ToySceneCfg = field(default_factory=ToySceneCfg)
    sim: ToySimCfg = field(default_factory=ToySimCfg)
    episode_length: int = 50


class ToyEnv:
    def __init__(self, cfg: ToyEnvCfg | None = None, render_mode=None, **kw):
        self.cfg = cfg or ToyEnvCfg()
        self.num_envs = self.cfg.scene.num_envs
        self.device = torch.device(self.cfg.sim.device)
        self.max_episode_length = self.cfg.episode_length
        self.episode_length_buf = torch.zeros(self.num_envs, dtype=torch.long)
        self.g = torch.Generator().manual_seed(self.cfg.seed or 0)
        self.x = torch.zeros(self.num_envs, 3)
        self.target = torch.zeros(self.num_envs, 3)
        self.action_manager = SimpleNamespace(total_action_dim=3)
        self.observation_manager = SimpleNamespace(group_obs_dim={"policy": (6,)}, compute=self._obs)
        self.render_mode = render_mode

    @property
    def unwrapped(self):
        return self

    def _obs(self):
        return {"policy": torch.cat([self.target - self.x, self.x], dim=1)}

    def _reset(self, ids):
        self.x[ids] = 0.0
        self.target[ids] = torch.rand(len(ids), 3, generator=self.g) * 2 - 1
        self.episode_length_buf[ids] = 0

    def reset(self, seed=None, options=None):
        self._reset(torch.arange(self.num_envs))
        return self._obs(), {}

    def step(self, a):
        self.x += 0.1 * a.clamp(-1, 1)
        rew = -(self.target - self.x).square().sum(dim=1)
        self.episode_length_buf += 1
        trunc = self.episode_length_buf >= self.max_episode_length
        term = torch.zeros_like(trunc)
        ids = trunc.nonzero().flatten()
        if len(ids):
            self._reset(ids)
        return self._obs(), rew, term, trunc, {"log": {"Episode_Reward/dist": rew.mean()}}

    def close(self):
        pass
