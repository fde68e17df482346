"""isaaclab_rl.rsl_rl: runner / policy / algorithm cfgs and RslRlVecEnvWrapper (IsaacLab 2.1 surface)."""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field

import torch

from isaaclab.utils.dict import class_to_dict


@dataclass
class RslRlPpoActorCriticCfg:
    class_name: str = "ActorCritic"
    init_noise_std: float = 1.0
    noise_std_type: str = "scalar"
    actor_hidden_dims: list = field(default_factory=lambda: [256, 256, 256])
    critic_hidden_dims: list = field(default_factory=lambda: [256, 256, 256])
    activation: str = "elu"


@dataclass
class RslRlPpoAlgorithmCfg:
    class_name: str = "PPO"
    num_learning_epochs: int = 5
    num_mini_batches: int = 4
    learning_rate: float = 1.0e-3
    schedule: str = "adaptive"
    gamma: float = 0.99
    lam: float = 0.95
    entropy_coef: float = 0.01
    desired_kl: float = 0.01
    max_grad_norm: float = 1.0
    value_loss_coef: float = 1.0
    use_clipped_value_loss: bool = True
    clip_param: float = 0.2
    normalize_advantage_per_mini_batch: bool = False
    symmetry_cfg: dict | None = None
    rnd_cfg: dict | None = None


@dataclass
class RslRlOnPolicyRunnerCfg:
    seed: int = 42
    device: str = "cuda:0"
    num_steps_per_env: int = 24
    max_iterations: int = 1500
    empirical_normalization: bool = False
    policy: RslRlPpoActorCriticCfg = field(default_factory=RslRlPpoActorCriticCfg)
    algorithm: RslRlPpoAlgorithmCfg = field(default_factory=RslRlPpoAlgorithmCfg)
    clip_actions: float | None = None
    save_interval: int = 50
    experiment_name: str = "default"
    run_name: str = ""
    logger: str = "tensorboard"
    neptune_project: str = "isaaclab"
    wandb_project: str = "isaaclab"
    resume: bool = False
    load_run: str = ".*"
    load_checkpoint: str = "model_.*.pt"

    def to_dict(self) -> dict:
        return class_to_dict(self)

    def replace(self, **kw):
        return dataclasses.replace(self, **kw)


class RslRlVecEnvWrapper:
    """Wraps the env for rsl_rl: obs tensor + {"observations": obs_dict} extras, long dones, time-outs."""

    def __init__(self, env, clip_actions: float | None = None):
        self.env = env
        self.clip_actions = clip_actions
        u = env.unwrapped
        self.num_envs = u.num_envs
        self.device = u.device
        self.max_episode_length = u.max_episode_length
        self.num_actions = u.action_manager.total_action_dim
        self.num_obs = u.observation_manager.group_obs_dim["policy"][0]
        crit = u.observation_manager.group_obs_dim.get("critic")
        self.num_privileged_obs = crit[0] if crit is not None else None
        self.shard = getattr(u, "shard", None)
        self.env.reset()

    def __str__(self):
        return f"<{type(self).__name__}{self.env}>"

    @property
    def cfg(self):
        return self.unwrapped.cfg

    @property
    def render_mode(self):
        return getattr(self.env, "render_mode", None)

    @property
    def observation_space(self):
        return getattr(self.env, "observation_space", None)

    @property
    def action_space(self):
        return getattr(self.env, "action_space", None)

    @classmethod
    def class_name(cls) -> str:
        return cls.__name__

    @property
    def unwrapped(self):
        return self.env.unwrapped

    @property
    def episode_length_buf(self) -> torch.Tensor:
        return self.unwrapped.episode_length_buf

    @episode_length_buf.setter
    def episode_length_buf(self, value: torch.Tensor):
        self.unwrapped.episode_length_buf = value

    def seed(self, seed: int = -1) -> int:
        return self.unwrapped.seed(seed)

    def get_observations(self):
        obs_dict = self.unwrapped.observation_manager.compute()
        return obs_dict["policy"], {"observations": obs_dict}

    def reset(self):
        obs_dict, _ = self.env.reset()
        return obs_dict["policy"], {"observations": obs_dict}

    def step(self, actions: torch.Tensor):
        if self.clip_actions is not None:
            actions = torch.clamp(actions, -self.clip_actions, self.clip_actions)
        obs_dict, rew, terminated, truncated, extras = self.env.step(actions)
        dones = (terminated | truncated).to(dtype=torch.long)
        extras["observations"] = obs_dict
        if not getattr(self.unwrapped.cfg, "is_finite_horizon", False):
            extras["time_outs"] = truncated
        return obs_dict["policy"], rew, dones, extras

    def close(self):
        return self.env.close()


def export_policy_as_jit(policy, normalizer, path: str, filename="policy.pt"):
    from h12env.export import export_policy_as_jit as f

    return f(policy, normalizer, path, filename)


def export_policy_as_onnx(policy, normalizer, path: str, filename="policy.onnx", verbose=False):
    from h12env.export import export_policy_as_onnx as f

    return f(policy, normalizer, path, filename, verbose)


__all__ = ["RslRlOnPolicyRunnerCfg", "RslRlPpoActorCriticCfg", "RslRlPpoAlgorithmCfg", "RslRlVecEnvWrapper",
           "export_policy_as_jit", "export_policy_as_onnx"]
