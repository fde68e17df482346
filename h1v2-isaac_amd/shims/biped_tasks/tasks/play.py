"""Play variant: 50 envs, observation noise off (IsaacLab *_PLAY cfg convention)."""
from dataclasses import dataclass

from h12env.cfg import H12FlatEnvCfg


@dataclass
class H12FlatEnvCfg_PLAY(H12FlatEnvCfg):
    def __post_init__(self):
        self.scene.num_envs = 50
        self.observations.policy.enable_corruption = False
