from h12env.ppo import OnPolicyRunner

__all__ = ["OnPolicyRunner"]
