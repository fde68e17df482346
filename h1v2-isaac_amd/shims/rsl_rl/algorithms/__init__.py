from h12env.ppo import PPO

__all__ = ["PPO"]
