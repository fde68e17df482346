"""isaaclab.envs: ManagerBasedRLEnv resolves to the MI355X env for the H1-2 velocity cfgs."""
from __future__ import annotations

from h12env.cfg import H12FlatEnvCfg

_CFG_TYPES: list[type] = [H12FlatEnvCfg]


class _CfgMeta(type):
    def __instancecheck__(cls, obj):
        return isinstance(obj, tuple(_CFG_TYPES))

    def __subclasscheck__(cls, sub):
        return issubclass(sub, tuple(_CFG_TYPES))


class ManagerBasedRLEnvCfg(metaclass=_CfgMeta):
    """isinstance(cfg, ManagerBasedRLEnvCfg) holds for the cfg types the MI355X env implements."""

    @staticmethod
    def register(cfg_type: type) -> type:
        _CFG_TYPES.append(cfg_type)
        return cfg_type


class DirectRLEnvCfg:
    pass


class DirectMARLEnvCfg:
    pass


class DirectMARLEnv:
    pass


class ManagerBasedRLEnv:
    """Factory with the IsaacLab constructor signature ManagerBasedRLEnv(cfg, render_mode=None)."""

    def __new__(cls, cfg=None, render_mode=None, **kwargs):
        from h12env.env import H12VelocityEnv

        if cfg is not None and not isinstance(cfg, tuple(_CFG_TYPES)):
            raise TypeError(f"no MI355X env implements cfg type {type(cfg).__name__}")
        return H12VelocityEnv(cfg, render_mode=render_mode, **kwargs)


ManagerBasedEnv = ManagerBasedRLEnv


def multi_agent_to_single_agent(env, state_as_observation: bool = False):
    raise NotImplementedError("multi-agent (DirectMARLEnv) tasks are not part of the MI355X build")


__all__ = ["ManagerBasedRLEnv", "ManagerBasedRLEnvCfg", "ManagerBasedEnv", "DirectRLEnvCfg", "DirectMARLEnv",
           "DirectMARLEnvCfg", "multi_agent_to_single_agent"]
