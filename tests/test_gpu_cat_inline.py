"""GPU: CaT's constraint probabilities applied inside step_kernel (cat_prob_inline, round 6: every block waits for the
last block's fold of the running maxima and the still list, then rescales its own envs' rewards) against the
two-kernel path (cat_prob_kernel after step_kernel; H12_CAT_INLINE=0 at handle creation), bit for bit: observation
rows, rewards, done flags (the probabilities), the constraint sums and swing heights, the episode log -- over steps
with resets and still envs (the no_move remap reads other blocks' rows), at the metric's 4096 envs and on a ragged
grid.  Both run the same fused rows.  The device's wait diagnostic stays clear (env.close raises otherwise).
Reference behaviour: biped_tasks/utils/cat/cat_env.py:95-193, constraint_manager.py:126-269."""
import os

import pytest
import torch

from h12env._abi import F as FIELDS

pytestmark = pytest.mark.gpu


def _make(n, inline):
    from h12env.cfg import H12CaTEnvCfg
    from h12env.env import H12VelocityEnv

    cfg = H12CaTEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    old = os.environ.get("H12_CAT_INLINE")
    os.environ["H12_CAT_INLINE"] = "1" if inline else "0"
    try:
        env = H12VelocityEnv(cfg)
    finally:
        if old is None:
            del os.environ["H12_CAT_INLINE"]
        else:
            os.environ["H12_CAT_INLINE"] = old
    env.reset()
    g = torch.Generator(device="cpu").manual_seed(n)
    env.episode_length_buf = torch.randint(env.max_episode_length - 20, env.max_episode_length, (n,), generator=g,
                                           dtype=torch.int32)
    return env


@pytest.mark.parametrize("n,steps", [(4096, 30), (300, 30), (8192, 200)])
def test_cat_inline_equals_two_kernel_path(gpu, n, steps):
    """(8192 envs: 256 blocks, one per CU -- the largest grid the inline path takes; 200 steps.)"""
    a_env, b_env = _make(n, True), _make(n, False)
    assert a_env.cat_inline and not b_env.cat_inline
    gen = torch.Generator(device="cpu").manual_seed(11)
    resets = 0
    for t in range(steps):
        # small actions on some envs keep them still under a zero command (no_move's remap)
        act = torch.randn(n, 12, generator=gen) * (0.02 if t % 3 == 0 else 0.4)
        act = act.to(gpu)
        oa, ra, ta, ua, ea = a_env.step(act)
        ob, rb, tb, ub, eb = b_env.step(act)
        assert torch.equal(oa["policy"], ob["policy"]), t
        assert torch.equal(ra, rb), t
        assert torch.equal(ta, tb), t
        assert torch.equal(ua, ub), t
        fa, fb = a_env._fstate, b_env._fstate
        for k in ("CSTR_SUM", "CSTR_P", "SWING_H"):
            o, c = FIELDS[k]
            assert torch.equal(fa[o:o + c], fb[o:o + c]), (t, k)
        la, lb = dict(ea["log"]), dict(eb["log"])
        assert la.keys() == lb.keys()
        for k in la:
            assert torch.equal(torch.as_tensor(la[k]), torch.as_tensor(lb[k])), (t, k)
        resets += int(ua.sum().item())
    assert resets > 0
    assert (ta > 0).float().mean() > 0.0  # probabilities are active
    a_env.close()
    b_env.close()
