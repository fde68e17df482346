"""GPU: step_kernel's fused observation assembly (FuseCtx: the shifted history stored by the helper waves during the
physics loop; the newest slot, refilled rows and frame_out after it; the episode-log folds deferred to
log_flush_kernel) against the two-kernel step path (obs_assemble_kernel; H12_FUSE_OBS=0 at handle creation), bit for
bit: observation rows, rewards, done flags and the episode log, over steps with resets.  Covers both fused variants --
the spread path (whole blocks; the shifted-row stores split over the physics steps after the first: 3 of 4, and 2 of 3
at decimation 3) and the after-the-loop path (the ragged last block of 37 / 300 envs) -- with and without the
self-contact wave (64 or 128 helper lanes), Flat (history 10), Rsl (history 6) and CaT (its kernels after step_kernel
rescale the reward and add their constraint statistics to the same deferred log partials); logs read right after
their step and 100+ steps later (after env.py's chunk flushes)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _make(cfg_fn, n, fuse, **kw):
    from h12env.env import H12VelocityEnv

    cfg = cfg_fn()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    if "decimation" in kw:
        cfg.decimation = kw["decimation"]
    if "self_collision" in kw:
        cfg.sim.self_collision = kw["self_collision"]
    old = os.environ.get("H12_FUSE_OBS")
    os.environ["H12_FUSE_OBS"] = "1" if fuse else "0"
    try:
        env = H12VelocityEnv(cfg)
    finally:
        if old is None:
            del os.environ["H12_FUSE_OBS"]
        else:
            os.environ["H12_FUSE_OBS"] = old
    env.reset()
    # episodes near their time-out: resets (refilled rows) inside the window, plus natural falls
    g = torch.Generator(device="cpu").manual_seed(n)
    env.episode_length_buf = torch.randint(env.max_episode_length - 30, env.max_episode_length, (n,), generator=g,
                                           dtype=torch.int32)
    return env


CASES = [
    ("flat", 256, {"steps": 140}),
    ("flat", 37, {}),
    ("flat", 300, {}),
    ("rsl", 64, {}),
    ("flat", 96, {"self_collision": False}),
    ("flat", 64, {"decimation": 3}),
    ("cat", 128, {}),
]


def _same_log(t, la, lb):
    la, lb = dict(la), dict(lb)
    assert la.keys() == lb.keys()
    for k in la:
        assert torch.equal(torch.as_tensor(la[k]), torch.as_tensor(lb[k])), (t, k)


@pytest.mark.parametrize("task,n,kw", CASES, ids=[f"{t}-{n}-{'-'.join(f'{k}{v}' for k, v in kw.items()) or 'default'}"
                                                  for t, n, kw in CASES])
def test_fused_assembly_equals_two_kernel_path(gpu, task, n, kw):
    from h12env import H12FlatEnvCfg
    from h12env.cfg import H12CaTEnvCfg, H12RslEnvCfg

    cfg_fn = {"flat": H12FlatEnvCfg, "rsl": H12RslEnvCfg, "cat": H12CaTEnvCfg}[task]
    kw = dict(kw)
    steps = kw.pop("steps", 40)
    a_env, b_env = _make(cfg_fn, n, True, **kw), _make(cfg_fn, n, False, **kw)
    assert torch.equal(a_env.get_observations()["policy"], b_env.get_observations()["policy"])
    gen = torch.Generator(device="cpu").manual_seed(3)
    resets = 0
    logs = []
    for t in range(steps):
        act = torch.randn(n, 12, generator=gen).to(gpu)
        oa, ra, ta, ua, ea = a_env.step(act)
        ob, rb, tb, ub, eb = b_env.step(act)
        pa, pb = oa["policy"], ob["policy"]
        assert torch.equal(pa.view(torch.int32), pb.view(torch.int32)), (t, (pa != pb).nonzero()[:5])
        # CaT returns the constraint termination probability as its dones
        assert torch.equal(ra, rb) and torch.equal(ta, tb) and torch.equal(ua, ub), t
        assert torch.equal(a_env.reset_terminated, b_env.reset_terminated), t
        resets += int((a_env.reset_terminated | a_env.reset_time_outs).sum())
        logs.append((ea["log"], eb["log"]))
        if t % 10 == 9:  # read now (a flush of the pending folds), the others at the end (deferred over >= 64 steps)
            _same_log(t, *logs[-1])
    for t, (la, lb) in enumerate(logs):
        _same_log(t, la, lb)
    assert resets > 0  # refilled rows were exercised
    a_env.close()
    b_env.close()
