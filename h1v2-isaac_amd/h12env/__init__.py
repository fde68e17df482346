"""h12env — MI355X-native vectorised H1-2 12-DoF velocity-tracking environment.

The hot path of `Isaac-Velocity-Flat-H12_12dof-v0` (reference: olivier-stasse/h1v2-Isaac) as one
fused HIP kernel per env step behind a C-ABI (include/h12env.h, libh12env.so), with a Python host
mirroring IsaacLab's ManagerBasedRLEnv surface.
"""
from .cfg import H12FlatEnvCfg, mujoco_cfg
from .model import body_names, build_model, joint_names

TASK_ID = "Isaac-Velocity-Flat-H12_12dof-v0"

__all__ = ["H12FlatEnvCfg", "mujoco_cfg", "build_model", "joint_names", "body_names", "TASK_ID", "make_env"]


def make_env(cfg: H12FlatEnvCfg | None = None, **kw):
    from .env import H12VelocityEnv

    return H12VelocityEnv(cfg, **kw)
