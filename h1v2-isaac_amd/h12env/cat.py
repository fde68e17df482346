"""`CaTEnv` (biped_tasks/utils/cat/cat_env.py:30-275) on the MI355X env: the Constraints-as-Terminations
variant of ``ManagerBasedRLEnv.step``.  The HIP path does the work (step_kernel computes the constraints,
cat_reduce_kernel / cat_prob_kernel the running maxima, probabilities, reward scaling and dones); this class
only names the entry point and requires a cfg with a ConstraintManager section."""
from __future__ import annotations

from .cfg import H12CaTEnvCfg
from .env import H12VelocityEnv


class CaTEnv(H12VelocityEnv):
    """step() -> (obs, reward * (1 - p), dones = p (1 where reset), time_outs, extras), cat_env.py:95-193."""

    def __init__(self, cfg: H12CaTEnvCfg | None = None, render_mode: str | None = None, **kwargs):
        cfg = cfg if cfg is not None else H12CaTEnvCfg()
        if getattr(cfg, "constraints", None) is None:
            raise ValueError("CaTEnv needs a cfg with constraints (H12CaTEnvCfg)")
        super().__init__(cfg, render_mode=render_mode, **kwargs)
