"""Task registration (mirrors biped_tasks/tasks/locomotion/velocity/config/h12_12dof/__init__.py:14-56
for the tasks this build implements; ids and entry-point keys unchanged)."""
import gymnasium as gym

from . import agents  # noqa: F401

gym.register(
    id="Isaac-Velocity-Rough-H12_12dof-v0",
    entry_point="isaaclab.envs:ManagerBasedRLEnv",
    disable_env_checker=True,
    kwargs={
        "env_cfg_entry_point": "h12env.cfg:H12RoughEnvCfg",
        "rsl_rl_cfg_entry_point": f"{agents.__name__}:H12_12dof_RoughPPORunnerCfg",
    },
)

gym.register(
    id="Isaac-Velocity-Rough-H12_12dof-Play-v0",
    entry_point="isaaclab.envs:ManagerBasedRLEnv",
    disable_env_checker=True,
    kwargs={
        "env_cfg_entry_point": "h12env.cfg:H12RoughEnvCfg_PLAY",
        "rsl_rl_cfg_entry_point": f"{agents.__name__}:H12_12dof_RoughPPORunnerCfg",
    },
)

gym.register(
    id="Isaac-Velocity-Flat-H12_12dof-v0",
    entry_point="isaaclab.envs:ManagerBasedRLEnv",
    disable_env_checker=True,
    kwargs={
        "env_cfg_entry_point": "h12env.cfg:H12FlatEnvCfg",
        "rsl_rl_cfg_entry_point": f"{agents.__name__}:H12_12dof_FlatPPORunnerCfg",
    },
)

gym.register(
    id="Isaac-Velocity-Flat-H12_12dof-Play-v0",
    entry_point="isaaclab.envs:ManagerBasedRLEnv",
    disable_env_checker=True,
    kwargs={
        "env_cfg_entry_point": f"{__name__}.play:H12FlatEnvCfg_PLAY",
        "rsl_rl_cfg_entry_point": f"{agents.__name__}:H12_12dof_FlatPPORunnerCfg",
    },
)

# h12_12dof/__init__.py:85-103: the Rsl task (IdealPD, deadzone commands, pushes, history 6; the task the
# shipped deploy env.yamls were exported from), trained with the Flat PPO runner cfg
gym.register(
    id="Isaac-Velocity-Rsl-H12_12dof-v0",
    entry_point="isaaclab.envs:ManagerBasedRLEnv",
    disable_env_checker=True,
    kwargs={
        "env_cfg_entry_point": "h12env.cfg:H12RslEnvCfg",
        "rsl_rl_cfg_entry_point": f"{agents.__name__}:H12_12dof_FlatPPORunnerCfg",
    },
)

gym.register(
    id="Isaac-Velocity-Rsl-H12_12dof-Play-v0",
    entry_point="isaaclab.envs:ManagerBasedRLEnv",
    disable_env_checker=True,
    kwargs={
        "env_cfg_entry_point": "h12env.cfg:H12RslEnvCfg_PLAY",
        "rsl_rl_cfg_entry_point": f"{agents.__name__}:H12_12dof_FlatPPORunnerCfg",
    },
)

# h12_12dof/__init__.py:64-83: Constraints-as-Terminations (the env class returns the constraint termination
# probability as dones; trained by the reference with CleanRL's PPO, which this build does not ship)
gym.register(
    id="Isaac-Velocity-CaT-Flat-H12_12dof-v0",
    entry_point="h12env.cat:CaTEnv",
    disable_env_checker=True,
    kwargs={"env_cfg_entry_point": "h12env.cfg:H12CaTEnvCfg"},
)

gym.register(
    id="Isaac-Velocity-CaT-Flat-H12_12dof-Play-v0",
    entry_point="h12env.cat:CaTEnv",
    disable_env_checker=True,
    kwargs={"env_cfg_entry_point": "h12env.cfg:H12CaTEnvCfg_PLAY"},
)
