from h12env.ppo import ActorCritic, EmpiricalNormalization

__all__ = ["ActorCritic", "EmpiricalNormalization"]
