"""PPO runner cfgs of the H1-2 12-DoF tasks (values of biped_tasks/.../h12_12dof/agents/rsl_rl_ppo_cfg.py:10-47)."""
from dataclasses import dataclass, field

from isaaclab_rl.rsl_rl import RslRlOnPolicyRunnerCfg, RslRlPpoActorCriticCfg, RslRlPpoAlgorithmCfg


@dataclass
class H12_12dof_RoughPPORunnerCfg(RslRlOnPolicyRunnerCfg):
    num_steps_per_env: int = 24
    max_iterations: int = 3000
    save_interval: int = 100
    experiment_name: str = "h12_12dof_rough"
    empirical_normalization: bool = False
    policy: RslRlPpoActorCriticCfg = field(default_factory=lambda: RslRlPpoActorCriticCfg(
        init_noise_std=1.0, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[512, 256, 128], activation="elu"))
    algorithm: RslRlPpoAlgorithmCfg = field(default_factory=lambda: RslRlPpoAlgorithmCfg(
        value_loss_coef=1.0, use_clipped_value_loss=True, clip_param=0.2, entropy_coef=0.0081, num_learning_epochs=5,
        num_mini_batches=4, learning_rate=1.0e-3, schedule="adaptive", gamma=0.99, lam=0.95, desired_kl=0.01,
        max_grad_norm=1.0))


@dataclass
class H12_12dof_FlatPPORunnerCfg(H12_12dof_RoughPPORunnerCfg):
    max_iterations: int = 3000
    experiment_name: str = "h12_12dof_flat"
