"""PPO runner for the H1-2 env: the rsl_rl 2.3 OnPolicyRunner surface that scripts/rsl_rl/train.py drives
(reference: scripts/rsl_rl/train.py:123-141; agent cfg biped_tasks/.../h12_12dof/agents/rsl_rl_ppo_cfg.py:10-47;
algorithm: rsl-rl-lib 2.3.3 as pinned in uv.lock, restated here -- the package is not importable offline).

Design for one process per MI355X:
  * the rollout lives in HBM as (T, N, ...) tensors filled in place; the env's observation buffer is
    copied into it once per step (the env keeps a ping-pong buffer);
  * multi-GPU (torchrun, one rank per GPU): each rank collects its env shard, the rollout is
    all-gathered over RCCL/xGMI in one collective per dtype bucket (h12env.distributed.allgather_rollout,
    the north_star's exchange), every rank draws the same minibatch permutation of the GLOBAL batch,
    computes gradients on its 1/world share of each minibatch, and the gradients are averaged with one
    flat all-reduce -- so all ranks apply bit-identical updates (parameters are also broadcast from rank 0
    at start and on load);
  * checkpoints use rsl_rl's layout ({"model_state_dict", "optimizer_state_dict", "iter", "infos"}).
"""
from __future__ import annotations

import json
import math
import os
import statistics
import subprocess
import time
from collections import deque
from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn as nn
from torch.distributions import Normal

from . import distributed as D


# ---------------------------------------------------------------------------------------------- modules
def activation(name: str) -> nn.Module:
    table = {"elu": nn.ELU, "selu": nn.SELU, "relu": nn.ReLU, "lrelu": nn.LeakyReLU, "tanh": nn.Tanh,
             "sigmoid": nn.Sigmoid, "gelu": nn.GELU}
    if name not in table:
        raise ValueError(f"unknown activation {name!r}")
    return table[name]()


class _SplitKLinearFn(torch.autograd.Function):
    """y = x W^T + b whose weight gradient dW = dY^T X is computed as SPLIT_K batched GEMMs over slices of the
    minibatch and summed: a (out x in) GEMM with K = 24576 gives hipBLASLt only ~17 output tiles for the 256
    CUs (measured 20 TFLOP/s); split 16 ways it runs 1.5x faster end to end (exp: fwd+bwd of both MLPs
    2.19 -> 1.48 ms per minibatch).  Same math, fp32 summation order differs.  dt: the GEMM operand type
    (float32, or bfloat16 under the bf16 learner's autocast: the partial products are summed in fp32 and the
    gradients of the fp32 master weights are fp32)."""

    @staticmethod
    def forward(ctx, x, w, b, split, dt):
        with torch.autocast(device_type="cuda", enabled=False):
            xc, wc = x.to(dt), w.to(dt)
            ctx.save_for_backward(xc, wc)
            ctx.split, ctx.x_dtype = split, x.dtype
            return torch.addmm(b.to(dt), xc, wc.t())

    @staticmethod
    def backward(ctx, gy):
        xc, wc = ctx.saved_tensors
        s, n = ctx.split, xc.shape[0]
        with torch.autocast(device_type="cuda", enabled=False):
            gy = gy.to(wc.dtype)
            gx = (gy @ wc).to(ctx.x_dtype) if ctx.needs_input_grad[0] else None
            gw = torch.bmm(gy.view(s, n // s, -1).transpose(1, 2), xc.view(s, n // s, -1))
            gw = gw.sum(0) if gw.dtype == torch.float32 else gw.float().sum(0)
            return gx, gw, gy.float().sum(0), None, None


class SplitKLinear(nn.Linear):
    """nn.Linear (same parameters / state dict) with the split-K weight gradient for large GPU batches
    (fp32, or bf16 operands under autocast)."""

    SPLIT_K = 16
    MIN_BATCH = 8192

    def forward(self, x):
        if (x.is_cuda and x.dim() == 2 and self.weight.dtype == torch.float32 and torch.is_grad_enabled()
                and x.shape[0] >= self.MIN_BATCH and x.shape[0] % self.SPLIT_K == 0):
            dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else torch.float32
            if x.dtype in (torch.float32, dt):
                return _SplitKLinearFn.apply(x, self.weight, self.bias, self.SPLIT_K, dt)
        return nn.functional.linear(x, self.weight, self.bias)


def mlp(n_in: int, hidden: list[int], n_out: int, act: str) -> nn.Sequential:
    layers: list[nn.Module] = []
    d = n_in
    for h in hidden:
        layers += [SplitKLinear(d, h), activation(act)]
        d = h
    layers.append(SplitKLinear(d, n_out))
    return nn.Sequential(*layers)


def plain_linear(module: nn.Module) -> nn.Module:
    """A copy of `module` with every SplitKLinear replaced by an nn.Linear holding the same parameters
    (for TorchScript / ONNX export)."""
    import copy

    m = copy.deepcopy(module)
    for name, child in list(m.named_children()):
        if isinstance(child, SplitKLinear):
            lin = nn.Linear(child.in_features, child.out_features, device=child.weight.device, dtype=child.weight.dtype)
            lin.load_state_dict(child.state_dict())
            setattr(m, name, lin)
        else:
            setattr(m, name, plain_linear(child))
    return m


class ActorCritic(nn.Module):
    """Gaussian policy with a state-independent std (rsl_rl ActorCritic, noise_std_type "scalar"/"log")."""

    is_recurrent = False

    def __init__(self, num_actor_obs: int, num_critic_obs: int, num_actions: int, actor_hidden_dims=(256, 256, 256),
                 critic_hidden_dims=(256, 256, 256), activation="elu", init_noise_std=1.0, noise_std_type="scalar",
                 **kwargs):
        super().__init__()
        self.actor = mlp(num_actor_obs, list(actor_hidden_dims), num_actions, activation)
        self.critic = mlp(num_critic_obs, list(critic_hidden_dims), 1, activation)
        self.noise_std_type = noise_std_type
        if noise_std_type == "scalar":
            self.std = nn.Parameter(init_noise_std * torch.ones(num_actions))
        elif noise_std_type == "log":
            self.log_std = nn.Parameter(torch.log(init_noise_std * torch.ones(num_actions)))
        else:
            raise ValueError(f"unknown noise_std_type {noise_std_type!r}")
        self.distribution: Normal | None = None
        Normal.set_default_validate_args(False)

    def _std(self, mean):
        s = self.std if self.noise_std_type == "scalar" else torch.exp(self.log_std)
        return s.expand_as(mean)

    def update_distribution(self, obs):
        mean = self.actor(obs)
        self.distribution = Normal(mean, self._std(mean))

    def act(self, obs, **kw):
        self.update_distribution(obs)
        return self.distribution.sample()

    def act_inference(self, obs):
        return self.actor(obs)

    def evaluate(self, critic_obs, **kw):
        return self.critic(critic_obs)

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)

    @property
    def action_mean(self):
        return self.distribution.mean

    @property
    def action_std(self):
        return self.distribution.stddev

    @property
    def entropy(self):
        return self.distribution.entropy().sum(dim=-1)

    def reset(self, dones=None):
        pass


class EmpiricalNormalization(nn.Module):
    """Running mean / variance normaliser (rsl_rl EmpiricalNormalization); statistics frozen in eval."""

    def __init__(self, shape, eps=1e-2, until=None):
        super().__init__()
        self.eps = eps
        self.until = until
        self.register_buffer("_mean", torch.zeros(shape).unsqueeze(0))
        self.register_buffer("_var", torch.ones(shape).unsqueeze(0))
        self.register_buffer("_std", torch.ones(shape).unsqueeze(0))
        self.register_buffer("count", torch.tensor(0, dtype=torch.long))

    def forward(self, x):
        if self.training:
            self.update(x)
        return (x - self._mean) / (self._std + self.eps)

    @torch.jit.unused
    def update(self, x):
        """Running update from one batch; under torch.distributed (world > 1) the batch is the union of
        every rank's shard, so all ranks keep identical statistics.  The shards' statistics are merged with
        Chan's parallel formula (global mean from sum n_r mean_r, then M2 = sum n_r (var_r + (mean_r - mean)^2)):
        no E[x^2] - mean^2 cancellation, so the merged variance is never negative.  Every call issues exactly two
        all-reduces on every rank: the union size rides in the first one (with the shards' weighted means), so
        ranks never disagree on which collectives run, whatever their local batch sizes.  The merge and the sample count
        use the device-side union size (no host sync per update)."""
        if self.until is not None and self.count >= self.until:
            return
        n = x.shape[0]
        var_x = torch.var(x, dim=0, unbiased=False, keepdim=True)
        mean_x = torch.mean(x, dim=0, keepdim=True)
        if torch.distributed.is_available() and torch.distributed.is_initialized() \
                and torch.distributed.get_world_size() > 1:
            s1 = torch.cat([mean_x * n, torch.full((1, 1), float(n), device=x.device, dtype=mean_x.dtype)], 1)
            D.all_reduce(s1)
            n_dev = s1[:, -1:]
            g_mean = s1[:, :-1] / n_dev
            m2 = (var_x + (mean_x - g_mean) ** 2) * n
            D.all_reduce(m2)
            m2 = m2 / n_dev
            # the union size stays on the device (no host sync, and no cache that a rank whose own batch size is
            # unchanged could keep while another rank's changes)
            self.count += n_dev.reshape(()).round().long()
            rate = n_dev / self.count
            mean_x, var_x = g_mean, m2
        else:
            self.count += n
            rate = n / self.count
        delta = mean_x - self._mean
        self._mean += rate * delta
        self._var += rate * (var_x - self._var + delta * (mean_x - self._mean))
        self._std = torch.sqrt(self._var)


# ---------------------------------------------------------------------------------------------- storage
class RolloutStorage:
    """(T, N, ...) device tensors of one PPO iteration (rsl_rl RolloutStorage, feed-forward case)."""

    def __init__(self, num_envs, num_steps, obs_dim, critic_obs_dim, num_actions, device):
        T, N = num_steps, num_envs
        self.num_envs, self.num_steps, self.device = N, T, device
        z = lambda *s: torch.zeros(*s, device=device)  # noqa: E731
        self.t = {
            "observations": z(T, N, obs_dim),
            "actions": z(T, N, num_actions),
            "rewards": z(T, N, 1),
            "dones": z(T, N, 1),
            "values": z(T, N, 1),
            "actions_log_prob": z(T, N, 1),
            "mu": z(T, N, num_actions),
            "sigma": z(T, N, num_actions),
            "returns": z(T, N, 1),
            "advantages": z(T, N, 1),
        }
        if critic_obs_dim is not None:
            self.t["privileged_observations"] = z(T, N, critic_obs_dim)
        self.step = 0

    def __getattr__(self, k):
        t = self.__dict__.get("t")
        if t is not None and k in t:
            return t[k]
        raise AttributeError(k)

    def add(self, obs, critic_obs, actions, rewards, dones, values, log_prob, mu, sigma):
        if self.step >= self.num_steps:
            raise OverflowError("rollout buffer overflow; call clear() before adding new transitions")
        s = self.step
        t = self.t
        t["observations"][s].copy_(obs)
        if "privileged_observations" in t and critic_obs is not None:
            t["privileged_observations"][s].copy_(critic_obs)
        t["actions"][s].copy_(actions)
        t["rewards"][s].copy_(rewards.view(-1, 1))
        t["dones"][s].copy_(dones.view(-1, 1))
        t["values"][s].copy_(values)
        t["actions_log_prob"][s].copy_(log_prob.view(-1, 1))
        t["mu"][s].copy_(mu)
        t["sigma"][s].copy_(sigma)
        self.step += 1

    def clear(self):
        self.step = 0

    def compute_returns(self, last_values, gamma, lam, normalize_advantage=True):
        """GAE(gamma, lambda) backwards over the T steps, bootstrapped by last_values."""
        t = self.t
        adv = 0
        for s in reversed(range(self.num_steps)):
            nxt = last_values if s == self.num_steps - 1 else t["values"][s + 1]
            not_done = 1.0 - t["dones"][s]
            delta = t["rewards"][s] + not_done * gamma * nxt - t["values"][s]
            adv = delta + not_done * gamma * lam * adv
            t["returns"][s] = adv + t["values"][s]
        t["advantages"].copy_(t["returns"] - t["values"])
        if normalize_advantage:
            a = t["advantages"]
            t["advantages"].copy_((a - a.mean()) / (a.std() + 1e-8))


# ---------------------------------------------------------------------------------------------- PPO
def enable_tunable_gemm():
    """PyTorch's TunableOp for the learner's GEMMs: the first call of each GEMM shape times the available
    hipBLASLt / rocBLAS solutions and keeps the fastest for the process (the minibatch shapes are fixed, so a few
    seconds once per run).  Round 4, C3 at 4096 envs, 2 runs each: learning 38.6 / 38.5 ms per iteration against 41.3
    / 40.8 ms with the default heuristics (profiles/r4/r4t_blas_tunableop_ab.txt).

    OPT-IN (H12_TUNABLEOP=1, or bench.py --mode train --tunableop): the selection is the fastest solution of a timing
    run, so it can differ between runs and between ranks -- two runs with the same seed are then not bit-reproducible
    (each rank's GEMMs may round differently), and the switch is process-wide (every GEMM in the process is tuned).
    With PYTORCH_TUNABLEOP_FILENAME set to an existing tuning table the recorded selections are reused with tuning
    off (reproducible); otherwise the table is written to the temp directory."""
    import tempfile

    t = torch.cuda.tunable
    if not t.is_enabled():
        fixed = os.environ.get("PYTORCH_TUNABLEOP_FILENAME")
        if fixed and os.path.exists(fixed):
            t.enable(True)
            t.tuning_enable(False)  # a checked tuning table: its selections, no timing runs
            t.read_file(fixed)
            return
        if not fixed:
            t.set_filename(os.path.join(tempfile.gettempdir(), f"h12env_tunableop_{os.getpid()}_%d.csv"))
        t.enable(True)
        t.tuning_enable(True)


class PPO:
    """Clipped-surrogate PPO with clipped value loss, entropy bonus and KL-adaptive learning rate
    (rsl_rl 2.3 algorithms/ppo.py semantics)."""

    def __init__(self, policy, num_learning_epochs=1, num_mini_batches=1, clip_param=0.2, gamma=0.998, lam=0.95,
                 value_loss_coef=1.0, entropy_coef=0.0, learning_rate=1e-3, max_grad_norm=1.0,
                 use_clipped_value_loss=True, schedule="fixed", desired_kl=0.01, device="cpu",
                 normalize_advantage_per_mini_batch=False, shard: D.Shard | None = None, precision: str = "fp32",
                 **kwargs):
        self.policy = policy.to(device)
        self.actor_critic = self.policy  # rsl_rl < 2.3 name
        self.device = device
        if str(device).startswith("cuda") and os.environ.get("H12_TUNABLEOP", "0") == "1":
            enable_tunable_gemm()
        # fused Adam (one kernel for all parameters) on the GPU with the learning rate as a device tensor, so
        # the KL-adaptive schedule runs on the device (no host sync per minibatch); plain Adam on CPU
        fused = str(device).startswith("cuda")
        self._lr_t = torch.tensor(float(learning_rate), device=device) if fused else None
        self.optimizer = torch.optim.Adam(self.policy.parameters(), lr=self._lr_t if fused else learning_rate,
                                          fused=fused, capturable=fused)
        self._graph = None
        self.learning_rate = learning_rate
        self.num_learning_epochs = num_learning_epochs
        self.num_mini_batches = num_mini_batches
        self.clip_param = clip_param
        self.gamma, self.lam = gamma, lam
        self.value_loss_coef, self.entropy_coef = value_loss_coef, entropy_coef
        self.max_grad_norm = max_grad_norm
        self.use_clipped_value_loss = use_clipped_value_loss
        self.schedule, self.desired_kl = schedule, desired_kl
        self.normalize_advantage_per_mini_batch = normalize_advantage_per_mini_batch
        self.shard = shard or D.Shard(0, 1, 0, 0)
        self.storage: RolloutStorage | None = None
        self._update_count = 0
        # "bf16": autocast the learning-phase forward/backward GEMMs to bf16 MFMA (the reference trains with
        # TF32 matmuls enabled on NVIDIA, train.py:70-71; gfx950 has no TF32); "fp32": exact fp32
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be fp32 or bf16, got {precision!r}")
        self.precision = precision

    def init_storage(self, num_envs, num_steps, obs_shape, critic_obs_shape, action_shape):
        self.storage = RolloutStorage(num_envs, num_steps, obs_shape[0],
                                      None if critic_obs_shape is None else critic_obs_shape[0], action_shape[0],
                                      self.device)

    # ---- collection
    def act(self, obs, critic_obs):
        if self._act_graph_ok(obs, critic_obs):
            return self._act_graphed(obs, critic_obs)
        self._obs, self._critic_obs = obs, critic_obs
        self._actions = self.policy.act(obs).detach()
        self._values = self.policy.evaluate(critic_obs).detach()
        self._log_prob = self.policy.get_actions_log_prob(self._actions).detach()
        self._mu = self.policy.action_mean.detach()
        self._sigma = self.policy.action_std.detach()
        return self._actions

    # ---- collection as a HIP graph: actor + critic forward, Gaussian sample, log-probability in one launch
    def _act_graph_ok(self, obs, critic_obs) -> bool:
        return (obs.is_cuda and not torch.is_grad_enabled() and os.environ.get("H12_PPO_GRAPH", "1") != "0"
                and not getattr(self.policy, "is_recurrent", False))

    def _act_body(self):
        mean = self.policy.actor(self._ga_obs)
        std = self.policy._std(mean)
        # mean + std * N(0, 1): the same Normal(mean, std) sample as distribution.sample(), from randn (capturable)
        actions = mean + std * torch.randn_like(mean)
        values = self.policy.critic(self._ga_cobs)
        log_prob = Normal(mean, std).log_prob(actions).sum(dim=-1)
        self._ga_out = (actions, values, log_prob, mean, std)

    def _act_graphed(self, obs, critic_obs):
        key = (tuple(obs.shape), tuple(critic_obs.shape), critic_obs is obs, obs.dtype)
        if getattr(self, "_ga", None) is None or self._ga_key != key:
            # normal (not inference) tensors throughout: the graph's RNG state is updated outside inference mode
            # the warm-up and capture consume exploration-noise draws: the generator state is put back after
            # them, so the replays draw the same noise sequence as the eager path (graph-safe philox offsets)
            rng_state = torch.cuda.get_rng_state(obs.device)
            with torch.inference_mode(False), torch.no_grad():
                self._ga_obs = torch.zeros(obs.shape, dtype=obs.dtype, device=obs.device)
                self._ga_cobs = (self._ga_obs if critic_obs is obs else
                                 torch.zeros(critic_obs.shape, dtype=critic_obs.dtype, device=obs.device))
                s = torch.cuda.Stream(device=obs.device)
                s.wait_stream(torch.cuda.current_stream(obs.device))
                with torch.cuda.stream(s):
                    for _ in range(2):
                        self._act_body()
                torch.cuda.current_stream(obs.device).wait_stream(s)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._act_body()
            torch.cuda.set_rng_state(rng_state, obs.device)
            self._ga, self._ga_key = g, key
        self._ga_obs.copy_(obs)
        if critic_obs is not obs:
            self._ga_cobs.copy_(critic_obs)
        self._ga.replay()
        self._obs, self._critic_obs = obs, critic_obs
        self._actions, self._values, self._log_prob, self._mu, self._sigma = self._ga_out
        return self._actions

    def process_env_step(self, rewards, dones, infos):
        r = rewards.clone().float()
        if "time_outs" in infos:  # bootstrap on time-outs (rsl_rl ppo.py)
            r += self.gamma * (self._values.squeeze(1) * infos["time_outs"].to(self.device).float())
        self.storage.add(self._obs, self._critic_obs if self.storage.t.get("privileged_observations") is not None else None,
                         self._actions, r, dones.float(), self._values, self._log_prob, self._mu, self._sigma)
        self.policy.reset(dones)

    def compute_returns(self, last_critic_obs):
        last_values = self.policy.evaluate(last_critic_obs).detach()
        # multi-GPU: advantages are normalised over the all-gathered global batch in _batch()
        self.storage.compute_returns(last_values, self.gamma, self.lam,
                                     normalize_advantage=not self.normalize_advantage_per_mini_batch
                                     and self.shard.world == 1)

    # ---- learning
    def _batch(self):
        """Flattened (T*N_global, ...) views of the (all-gathered) rollout."""
        st = self.storage.t
        if self.shard.world > 1:
            keys = [k for k in st if k not in ("rewards", "dones")]
            g = D.allgather_rollout({k: st[k] for k in keys}, self.shard, env_dim=1)
            if not self.normalize_advantage_per_mini_batch:
                a = g["advantages"]
                g["advantages"] = (a - a.mean()) / (a.std() + 1e-8)
        else:
            g = st
        return {k: v.reshape(-1, *v.shape[2:]) for k, v in g.items() if k not in ("rewards", "dones")}

    def _allreduce_grads(self):
        if self.shard.world == 1:
            return
        grads = [p.grad for p in self.policy.parameters() if p.grad is not None]
        flat = torch.cat([g.reshape(-1) for g in grads])
        D.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat /= self.shard.world
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n

    def _minibatch(self, b: dict, idx: torch.Tensor, stats: torch.Tensor):
        """One PPO minibatch update (rsl_rl ppo.py update loop body): gather, forward, KL-adaptive learning
        rate, clipped surrogate + clipped value loss, backward, (all-reduce), grad clip, Adam, statistics.
        Host-sync free on the fused path, so it is also the body of the captured HIP graph."""
        world = self.shard.world
        obs = b["observations"][idx]
        critic_obs = b["privileged_observations"][idx] if "privileged_observations" in b else obs
        actions = b["actions"][idx]
        target_values = b["values"][idx]
        advantages = b["advantages"][idx]
        returns = b["returns"][idx]
        old_log_prob = b["actions_log_prob"][idx]
        old_mu, old_sigma = b["mu"][idx], b["sigma"][idx]
        if self.normalize_advantage_per_mini_batch:
            advantages = (advantages - advantages.mean()) / (advantages.std() + 1e-8)
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16, cache_enabled=False,
                            enabled=self.precision == "bf16" and str(self.device).startswith("cuda")):
            self.policy.update_distribution(obs)  # rsl_rl calls act(); the sample itself is unused
            value = self.policy.evaluate(critic_obs).float()
        if self.precision == "bf16":  # distribution statistics in fp32
            self.policy.distribution = Normal(self.policy.distribution.mean.float(),
                                              self.policy.distribution.stddev.float())
        log_prob = self.policy.get_actions_log_prob(actions)
        mu, sigma, entropy = self.policy.action_mean, self.policy.action_std, self.policy.entropy
        if self.desired_kl is not None and self.schedule == "adaptive":
            with torch.no_grad():
                kl = torch.sum(torch.log(sigma / old_sigma + 1e-5)
                               + (old_sigma.square() + (old_mu - mu).square()) / (2.0 * sigma.square()) - 0.5, dim=-1)
                kl_mean = kl.mean()
                if world > 1:
                    D.all_reduce(kl_mean, op=dist.ReduceOp.SUM)
                    kl_mean /= world
                if self._lr_t is not None:
                    # rsl_rl's schedule on the device tensor the fused optimizer reads
                    lr = self._lr_t
                    up = kl_mean > self.desired_kl * 2.0
                    down = (kl_mean > 0.0) & (kl_mean < self.desired_kl / 2.0)
                    self._lr_t.copy_(torch.where(up, torch.clamp(lr / 1.5, min=1e-5),
                                                 torch.where(down, torch.clamp(lr * 1.5, max=1e-2), lr)))
                else:
                    k = kl_mean.item()
                    if k > self.desired_kl * 2.0:
                        self.learning_rate = max(1e-5, self.learning_rate / 1.5)
                    elif 0.0 < k < self.desired_kl / 2.0:
                        self.learning_rate = min(1e-2, self.learning_rate * 1.5)
                    for g in self.optimizer.param_groups:
                        g["lr"] = self.learning_rate
        ratio = torch.exp(log_prob - old_log_prob.squeeze(-1))
        adv = advantages.squeeze(-1)
        surrogate = -adv * ratio
        surrogate_clipped = -adv * torch.clamp(ratio, 1.0 - self.clip_param, 1.0 + self.clip_param)
        surrogate_loss = torch.max(surrogate, surrogate_clipped).mean()
        if self.use_clipped_value_loss:
            v_clipped = target_values + (value - target_values).clamp(-self.clip_param, self.clip_param)
            value_loss = torch.max((value - returns).square(), (v_clipped - returns).square()).mean()
        else:
            value_loss = (returns - value).square().mean()
        loss = surrogate_loss + self.value_loss_coef * value_loss - self.entropy_coef * entropy.mean()
        self.optimizer.zero_grad(set_to_none=True)  # backward writes the grads (no fill + add)
        loss.backward()
        self._allreduce_grads()
        nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm)
        self.optimizer.step()
        stats += torch.stack([value_loss.detach(), surrogate_loss.detach(), entropy.mean().detach()])

    def _graph_ok(self) -> bool:
        return (self._lr_t is not None and self.shard.world == 1 and str(self.device).startswith("cuda")
                and os.environ.get("H12_PPO_GRAPH", "1") != "0")

    def _snapshot(self):
        st = {}
        for p in self.policy.parameters():
            st[p] = {k: v.detach().clone() for k, v in self.optimizer.state.get(p, {}).items() if torch.is_tensor(v)}
        return [p.detach().clone() for p in self.policy.parameters()], st, self._lr_t.clone()

    def _restore(self, snap):
        params, st, lr = snap
        with torch.no_grad():
            for p, v in zip(self.policy.parameters(), params):
                p.copy_(v)
            for p in self.policy.parameters():
                for k, v in self.optimizer.state.get(p, {}).items():
                    if torch.is_tensor(v):
                        v.copy_(st[p][k]) if k in st[p] else v.zero_()  # lazily created by the warm-up: initial 0
            self._lr_t.copy_(lr)

    def _capture(self, b: dict, mb: int):
        """Capture one minibatch update as a HIP graph (replayed num_epochs x num_mini_batches times per
        update): the ~300 kernel launches of a minibatch cost one graph launch.  Warm-up runs on a side
        stream on the real parameters, which are restored bit-exactly before the capture."""
        self._g_idx = torch.zeros(mb, dtype=torch.long, device=self.device)
        self._g_stats = torch.zeros(3, device=self.device)
        self.policy.distribution = None  # drop autograd graphs built on the default stream
        snap = self._snapshot()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):
                self._minibatch(b, self._g_idx, self._g_stats)
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.policy.distribution = None
        self._restore(snap)
        self._g_stats.zero_()
        g = torch.cuda.CUDAGraph()
        self.optimizer.zero_grad(set_to_none=True)
        with torch.cuda.graph(g):
            self._minibatch(b, self._g_idx, self._g_stats)
        self._graph = g
        self._graph_key = (mb, tuple((k, v.data_ptr(), tuple(v.shape)) for k, v in sorted(b.items())))

    def update(self):
        b = self._batch()
        n_total = b["observations"].shape[0]
        mb = n_total // self.num_mini_batches
        world, rank = self.shard.world, self.shard.rank
        gen = torch.Generator(device=self.device)
        use_graph = self._graph_ok()
        if use_graph:
            key = (mb, tuple((k, v.data_ptr(), tuple(v.shape)) for k, v in sorted(b.items())))
            if getattr(self, "_graph", None) is None or self._graph_key != key:
                self._capture(b, mb)
            stats = self._g_stats
            stats.zero_()
        else:
            stats = torch.zeros(3, device=self.device)
        n_updates = 0
        for epoch in range(self.num_learning_epochs):
            # identical permutation on every rank (shared seed per epoch); each rank takes its share
            gen.manual_seed(1_000_003 * self._update_count + epoch)
            perm = torch.randperm(n_total, generator=gen, device=self.device)
            for i in range(self.num_mini_batches):
                idx = perm[i * mb:(i + 1) * mb]
                if world > 1:
                    share = mb // world
                    idx = idx[rank * share:(rank + 1) * share]
                if use_graph:
                    self._g_idx.copy_(idx)
                    self._graph.replay()
                else:
                    self._minibatch(b, idx, stats)
                n_updates += 1
        self._update_count += 1
        self.storage.clear()
        if self._lr_t is not None:
            self.learning_rate = float(self._lr_t)
        v, sl, en = (stats / n_updates).tolist()
        return {"value_function": v, "surrogate": sl, "entropy": en}

    def optimizer_state_dict(self) -> dict:
        """The optimizer state with a plain-float learning rate (rsl_rl's checkpoint layout)."""
        sd = self.optimizer.state_dict()
        for g in sd["param_groups"]:
            if torch.is_tensor(g["lr"]):
                g["lr"] = float(g["lr"])
        return sd

    def load_optimizer_state_dict(self, sd: dict):
        self.optimizer.load_state_dict(sd)
        self._graph = None  # the captured graph holds the old state tensors
        lr = float(self.optimizer.param_groups[0]["lr"])
        self.learning_rate = lr
        if self._lr_t is not None:  # keep the device tensor the schedule updates in the param groups
            self._lr_t.fill_(lr)
            for g in self.optimizer.param_groups:
                g["lr"] = self._lr_t

    def broadcast_parameters(self):
        if self.shard.world > 1:
            for p in self.policy.state_dict().values():
                D.broadcast(p, src=0)


# ---------------------------------------------------------------------------------------------- runner
@dataclass
class _Logger:
    log_dir: str | None
    rank: int

    def __post_init__(self):
        self._fh = None

    def write(self, it: int, scalars: dict):
        # the run directory is created lazily (a resume looks up the previous run before this one exists)
        if self._fh is None and self.log_dir and self.rank == 0:
            os.makedirs(self.log_dir, exist_ok=True)
            self._fh = open(os.path.join(self.log_dir, "metrics.jsonl"), "a")
        if self._fh:
            self._fh.write(json.dumps({"iter": it, **scalars}) + "\n")
            self._fh.flush()

    def close(self):
        if self._fh:
            self._fh.close()
            self._fh = None


class OnPolicyRunner:
    """rsl_rl 2.3 OnPolicyRunner: collect num_steps_per_env transitions from every env, PPO update,
    log, checkpoint every save_interval iterations."""

    def __init__(self, env, train_cfg: dict, log_dir: str | None = None, device="cpu"):
        self.cfg = train_cfg
        self.alg_cfg = dict(train_cfg["algorithm"])
        self.policy_cfg = dict(train_cfg["policy"])
        self.device = device
        self.env = env
        self.shard = getattr(env, "shard", None) or _shard_from_env()
        # learner RNG per rank (IsaacLab's distributed train.py: seed + local rank), so the exploration noise
        # and init_at_random_ep_len draws differ between shards; parameters are broadcast from rank 0 below.
        # The env's own streams stay keyed by the global env id (shard-invariant trajectories).
        seed = int(train_cfg.get("seed", 1))
        torch.manual_seed(seed + self.shard.rank)
        obs, extras = env.get_observations()
        num_obs = obs.shape[1]
        critic_obs = extras["observations"].get("critic")
        num_critic_obs = critic_obs.shape[1] if critic_obs is not None else num_obs
        self.policy_cfg.pop("class_name", None)
        policy = ActorCritic(num_obs, num_critic_obs, env.num_actions, **self.policy_cfg).to(device)
        self.alg_cfg.pop("class_name", None)
        self.alg_cfg.pop("rnd_cfg", None)
        self.alg_cfg.pop("symmetry_cfg", None)
        self.alg = PPO(policy, device=device, shard=self.shard, **self.alg_cfg)
        self.alg.broadcast_parameters()
        self.num_steps_per_env = int(train_cfg["num_steps_per_env"])
        self.save_interval = int(train_cfg.get("save_interval", 50))
        self.empirical_normalization = bool(train_cfg.get("empirical_normalization", False))
        if self.empirical_normalization:
            self.obs_normalizer = EmpiricalNormalization([num_obs], until=1.0e8).to(device)
            self.critic_obs_normalizer = EmpiricalNormalization([num_critic_obs], until=1.0e8).to(device)
        else:
            self.obs_normalizer = nn.Identity().to(device)
            self.critic_obs_normalizer = nn.Identity().to(device)
        self.alg.init_storage(env.num_envs, self.num_steps_per_env, [num_obs],
                              None if critic_obs is None else [num_critic_obs], [env.num_actions])
        self.log_dir = log_dir
        self.logger = _Logger(log_dir, self.shard.rank)
        self.tot_timesteps = 0
        self.tot_time = 0.0
        self.current_learning_iteration = 0
        self.git_status_repos: list[str] = []
        self.last_iteration_stats: dict = {}
        self.env.reset()

    # ---- API used by train.py / play.py
    def learn(self, num_learning_iterations: int, init_at_random_ep_len: bool = False):
        if init_at_random_ep_len:
            self.env.episode_length_buf = torch.randint_like(self.env.episode_length_buf,
                                                             high=int(self.env.max_episode_length))
        obs, extras = self.env.get_observations()
        critic_obs = extras["observations"].get("critic", obs)
        obs, critic_obs = obs.to(self.device), critic_obs.to(self.device)
        self.train_mode()
        self._store_git_state()
        ep_infos: list[dict] = []
        rewbuffer, lenbuffer = deque(maxlen=100), deque(maxlen=100)
        cur_reward_sum = torch.zeros(self.env.num_envs, device=self.device)
        cur_episode_length = torch.zeros(self.env.num_envs, device=self.device)
        done_mask: list = []
        done_rew: list = []
        done_len: list = []
        start_iter = self.current_learning_iteration
        self._start_iter = start_iter
        tot_iter = start_iter + num_learning_iterations
        for it in range(start_iter, tot_iter):
            start = time.time()
            with torch.inference_mode():
                for _ in range(self.num_steps_per_env):
                    actions = self.alg.act(obs, critic_obs)
                    obs, rewards, dones, infos = self.env.step(actions.to(self.env.device))
                    obs, rewards, dones = obs.to(self.device), rewards.to(self.device), dones.to(self.device)
                    obs = self.obs_normalizer(obs)
                    critic_obs = infos["observations"].get("critic", obs)
                    critic_obs = self.critic_obs_normalizer(critic_obs.to(self.device))
                    self.alg.process_env_step(rewards, dones, infos)
                    if self.log_dir is not None:
                        if "episode" in infos:
                            ep_infos.append(infos["episode"])
                        elif "log" in infos:
                            ep_infos.append(infos["log"])
                        # rsl_rl extends the reward / length deques at every step (a host sync per step);
                        # the finished episodes are recorded on the device and moved once per iteration,
                        # in the same order (step-major, env index within a step)
                        cur_reward_sum += rewards
                        cur_episode_length += 1
                        done = dones > 0
                        done_mask.append(done)
                        done_rew.append(torch.where(done, cur_reward_sum, 0.0))
                        done_len.append(torch.where(done, cur_episode_length, 0.0))
                        cur_reward_sum.masked_fill_(done, 0.0)
                        cur_episode_length.masked_fill_(done, 0.0)
                if self.log_dir is not None and done_mask:
                    m = torch.stack(done_mask)
                    rewbuffer.extend(torch.stack(done_rew)[m].cpu().tolist())
                    lenbuffer.extend(torch.stack(done_len)[m].cpu().tolist())
                    done_mask.clear()
                    done_rew.clear()
                    done_len.clear()
                stop = time.time()
                collection_time = stop - start
                start = stop
                self.alg.compute_returns(critic_obs)
            loss = self.alg.update()
            stop = time.time()
            learn_time = stop - start
            self.current_learning_iteration = it
            self._log(it, tot_iter, collection_time, learn_time, loss, ep_infos, rewbuffer, lenbuffer)
            if self.log_dir is not None and it % self.save_interval == 0:
                self.save(os.path.join(self.log_dir, f"model_{it}.pt"))
            ep_infos.clear()
        self.current_learning_iteration = tot_iter
        if self.log_dir is not None:
            self.save(os.path.join(self.log_dir, f"model_{self.current_learning_iteration}.pt"))

    def _log(self, it, tot_iter, collection_time, learn_time, loss, ep_infos, rewbuffer, lenbuffer):
        steps = self.num_steps_per_env * self.env.num_envs * self.shard.world
        self.tot_timesteps += steps
        it_time = collection_time + learn_time
        self.tot_time += it_time
        fps = int(steps / it_time) if it_time > 0 else 0
        scalars = {"Loss/value_function": loss["value_function"], "Loss/surrogate": loss["surrogate"],
                   "Loss/entropy": loss["entropy"], "Loss/learning_rate": self.alg.learning_rate,
                   "Policy/mean_noise_std": self.alg.policy.action_std.mean().item()
                   if self.alg.policy.distribution is not None else 0.0,
                   "Perf/total_fps": fps, "Perf/collection_time": collection_time, "Perf/learning_time": learn_time,
                   "Perf/collection_env_steps_per_s": self.env.num_envs * self.shard.world * self.num_steps_per_env
                   / max(collection_time, 1e-9)}
        for key in (ep_infos[0].keys() if ep_infos else []):
            vals = [float(torch.as_tensor(e[key]).float().mean()) for e in ep_infos if key in e]
            if vals:
                scalars[key if "/" in key else "Episode/" + key] = sum(vals) / len(vals)
        if rewbuffer:
            scalars["Train/mean_reward"] = statistics.mean(rewbuffer)
            scalars["Train/mean_episode_length"] = statistics.mean(lenbuffer)
        self.last_iteration_stats = scalars
        if self.shard.rank != 0:
            return
        self.logger.write(it, scalars)
        width = 80
        lines = [f"{'#' * width}", f" \033[1m Learning iteration {it}/{tot_iter} \033[0m ".center(width, " "),
                 f"{'Computation:':>35} {fps:.0f} steps/s (collection: {collection_time:.3f}s, learning {learn_time:.3f}s)"]
        for k, v in scalars.items():
            if not k.startswith("Perf/"):
                lines.append(f"{k + ':':>35} {v:.4f}")
        eta = self.tot_time / max(1, it + 1 - self._start_iter) * (tot_iter - it - 1)
        lines += [f"{'-' * width}", f"{'Total timesteps:':>35} {self.tot_timesteps}",
                  f"{'Iteration time:':>35} {it_time:.2f}s", f"{'Total time:':>35} {self.tot_time:.2f}s",
                  f"{'ETA:':>35} {eta:.1f}s"]
        print("\n".join(lines), flush=True)

    def save(self, path: str, infos=None):
        if self.shard.rank != 0:
            return
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        d = {"model_state_dict": self.alg.policy.state_dict(), "optimizer_state_dict": self.alg.optimizer_state_dict(),
             "iter": self.current_learning_iteration, "infos": infos}
        if self.empirical_normalization:
            d["obs_norm_state_dict"] = self.obs_normalizer.state_dict()
            d["critic_obs_norm_state_dict"] = self.critic_obs_normalizer.state_dict()
        torch.save(d, path)

    def load(self, path: str, load_optimizer: bool = True):
        d = torch.load(path, map_location=self.device, weights_only=True)
        self.alg.policy.load_state_dict(d["model_state_dict"])
        if self.empirical_normalization and "obs_norm_state_dict" in d:
            self.obs_normalizer.load_state_dict(d["obs_norm_state_dict"])
            self.critic_obs_normalizer.load_state_dict(d["critic_obs_norm_state_dict"])
        if load_optimizer and "optimizer_state_dict" in d:
            self.alg.load_optimizer_state_dict(d["optimizer_state_dict"])
        self.current_learning_iteration = int(d.get("iter", 0))
        self.alg.broadcast_parameters()
        return d.get("infos")

    def get_inference_policy(self, device=None):
        self.eval_mode()
        if device is not None:
            self.alg.policy.to(device)
        policy = self.alg.policy.act_inference
        if self.empirical_normalization:
            if device is not None:
                self.obs_normalizer.to(device)
            norm = self.obs_normalizer
            return lambda x: self.alg.policy.act_inference(norm(x))
        return policy

    def train_mode(self):
        self.alg.policy.train()
        if self.empirical_normalization:
            self.obs_normalizer.train()
            self.critic_obs_normalizer.train()

    def eval_mode(self):
        self.alg.policy.eval()
        if self.empirical_normalization:
            self.obs_normalizer.eval()
            self.critic_obs_normalizer.eval()

    def add_git_repo_to_log(self, repo_file_path):
        self.git_status_repos.append(repo_file_path)

    def _store_git_state(self):
        if self.log_dir is None or self.shard.rank != 0:
            return
        for p in self.git_status_repos:
            self._store_git_diff(p)
        self.git_status_repos = []

    def _store_git_diff(self, repo_file_path):
        try:
            d = os.path.dirname(os.path.abspath(repo_file_path))
            diff = subprocess.run(["git", "-C", d, "diff", "HEAD"], capture_output=True, text=True, timeout=10).stdout
            os.makedirs(self.log_dir, exist_ok=True)
            with open(os.path.join(self.log_dir, "git.diff"), "a") as f:
                f.write(f"--- {repo_file_path}\n{diff}\n")
        except Exception:  # not a git checkout: nothing to record
            pass


def _shard_from_env() -> D.Shard:
    if dist.is_available() and dist.is_initialized():
        return D.Shard(dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", "0")), 0)
    return D.Shard(0, 1, 0, 0)
