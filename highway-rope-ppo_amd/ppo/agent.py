"""PPO actor-critic for the MI355X build.

API-compatible with the reference's ppo/agent.py:
  * ActorCritic (:12-84): same module tree and parameter names (``shared.{0,2}``,
    ``actor_mean.{0,2}``, ``log_std``, ``critic.{0,2}``) so checkpoints load both ways;
    tanh-squashed Gaussian with the ``log1p(-a^2 + 1e-6)`` correction and the pre-tanh entropy.
  * PPOMemory (:87-154): list memory with store / clear / compute_advantages / get_batches /
    get_tensors; GAE runs in the HIP kernel (hwy_gae) with the reference's float64 arithmetic.
  * PPOAgent (:157-327): same constructor, select_action, update(last_value), save / load and
    the same metrics dict.

MI355X additions (the batched hot path):
  * ActorCritic.act(states) -- batched sampling on device, no host sync.
  * RolloutBuffer -- device-resident [T, E] rollout storage written by the env kernel in place.
  * PPOAgent.update_rollout(buffer, last_values) -- GAE kernel, global advantage normalisation,
    one minibatch permutation reused for every epoch (ppo/agent.py:205), per-minibatch clipped
    PPO step.  The step is captured once in a HIP graph and replayed; with a process group the
    flat gradient bucket is all-reduced (RCCL) between the two captured halves.
"""

from __future__ import annotations

import logging
import math
from typing import Any, Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Normal

from utils.graphs import capture as graph_capture

METRIC_KEYS = ("policy_loss", "value_loss", "entropy", "loss", "clip_fraction", "approx_kl")
_LOG_SQRT_2PI = 0.5 * math.log(2 * math.pi)


class ActorCritic(nn.Module):
    """Shared 2-layer ReLU trunk, actor mean head + state-independent log_std, critic head."""

    def __init__(self, state_dim: int, action_dim: int, hidden_dim: int = 128,
                 device: torch.device = torch.device("cpu")):
        super().__init__()
        self.device = device
        self.shared = nn.Sequential(
            nn.Linear(state_dim, hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, hidden_dim), nn.ReLU(),
        )
        self.actor_mean = nn.Sequential(
            nn.Linear(hidden_dim, hidden_dim), nn.ReLU(), nn.Linear(hidden_dim, action_dim)
        )
        self.log_std = nn.Parameter(torch.zeros(action_dim))
        self.critic = nn.Sequential(
            nn.Linear(hidden_dim, hidden_dim), nn.ReLU(), nn.Linear(hidden_dim, 1)
        )
        self.to(self.device)

    def forward(self, x):
        if isinstance(x, np.ndarray):
            x = torch.as_tensor(x, dtype=torch.float32, device=self.device)
        h = self.shared(x)
        return self.actor_mean(h), self.log_std.exp(), self.critic(h)

    @staticmethod
    def squashed_log_prob(dist: Normal, z: torch.Tensor) -> torch.Tensor:
        a = torch.tanh(z)
        return (dist.log_prob(z) - torch.log1p(-a.pow(2) + 1e-6)).sum(dim=-1)

    def get_action(self, state, deterministic: bool = False):
        """Reference single-state API (numpy in, numpy / Python scalars out)."""
        mean, std, value = self.forward(state)
        if deterministic:
            z = mean
            log_prob = None
        else:
            dist = Normal(mean, std, validate_args=False)
            z = dist.sample()
            log_prob = self.squashed_log_prob(dist, z)
        action = torch.tanh(z)
        return (action.detach().cpu().numpy(), z.detach().cpu().numpy(),
                None if log_prob is None else log_prob.item(),
                value.detach().cpu().numpy()[0])

    @torch.no_grad()
    def act(self, states: torch.Tensor, deterministic: bool = False,
            generator: Optional[torch.Generator] = None, noise: Optional[torch.Tensor] = None):
        """Batched device sampling: returns (action, pre_tanh, log_prob, value) tensors.
        ``noise`` (same shape as the mean) is a pre-drawn standard normal sample to use instead
        of drawing one from ``generator``."""
        mean, std, value = self.forward(states)
        if deterministic:
            z = mean
            logp = torch.zeros(mean.shape[0], device=mean.device)
        else:
            eps = noise if noise is not None else torch.randn(
                mean.shape, device=mean.device, dtype=mean.dtype, generator=generator)
            z = mean + std * eps
            logp = self.squashed_log_prob(Normal(mean, std, validate_args=False), z)
        return torch.tanh(z), z, logp, value.squeeze(-1)

    def evaluate(self, states, actions, pre_tanh_actions):
        mean, std, values = self.forward(states)
        dist = Normal(mean, std, validate_args=False)  # no host-syncing argument checks
        log_probs = self.squashed_log_prob(dist, pre_tanh_actions)
        entropy = dist.entropy().sum(dim=-1)
        return log_probs, values, entropy


class PPOMemory:
    """List-based rollout memory of the reference (one env, Python-side appends)."""

    def __init__(self, batch_size: int = 64, device: torch.device = torch.device("cpu")):
        self.batch_size = batch_size
        self.device = device
        self.clear()

    def store(self, state, action, pre_tanh_action, reward, next_state, log_prob, done, value):
        self.states.append(state)
        self.actions.append(action)
        self.pre_tanh_actions.append(pre_tanh_action)
        self.rewards.append(reward)
        self.next_states.append(next_state)
        self.log_probs.append(log_prob)
        self.dones.append(done)
        self.values.append(value)

    def clear(self):
        self.states: List[Any] = []
        self.actions: List[Any] = []
        self.pre_tanh_actions: List[Any] = []
        self.rewards: List[float] = []
        self.next_states: List[Any] = []
        self.log_probs: List[float] = []
        self.dones: List[bool] = []
        self.values: List[float] = []

    def compute_advantages(self, gamma: float, lam: float, last_value: float):
        """GAE of ppo/agent.py:126-138 on the HIP device (hwy_gae); returns numpy arrays."""
        from hwy import ops
        from hwy.native import HwyNativeError

        dev = self.device if torch.device(self.device).type == "cuda" else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None)
        if dev is None:
            raise HwyNativeError("compute_advantages runs the HIP GAE kernel; no HIP device found")
        T = len(self.rewards)
        rew = torch.as_tensor(np.asarray(self.rewards, np.float32).reshape(T, 1), device=dev)
        val = torch.as_tensor(np.asarray(self.values, np.float32).reshape(T, 1), device=dev)
        done = torch.as_tensor(np.asarray(self.dones, np.uint8).reshape(T, 1), device=dev)
        last = torch.tensor([float(last_value)], dtype=torch.float32, device=dev)
        adv, ret = ops.gae(rew, done, val, last, gamma, lam)
        return adv.view(T).cpu().numpy(), ret.view(T).cpu().numpy()

    def get_batches(self):
        n = len(self.states)
        indices = np.arange(n, dtype=np.int64)
        np.random.shuffle(indices)  # global numpy RNG, as ppo/agent.py:143
        return [indices[i:i + self.batch_size] for i in range(0, n, self.batch_size)]

    def get_tensors(self):
        dev = self.device
        f = lambda xs: torch.as_tensor(np.array(xs), dtype=torch.float32, device=dev)  # noqa: E731
        return f(self.states), f(self.actions), f(self.pre_tanh_actions), f(self.log_probs)


class RolloutBuffer:
    """Device-resident rollout of T steps x E envs (the env kernel writes rows in place)."""

    def __init__(self, T: int, E: int, state_dim: int, action_dim: int, device: torch.device):
        kw = dict(device=device, dtype=torch.float32)
        self.T, self.E, self.state_dim = T, E, state_dim
        self.states = torch.zeros(T + 1, E, state_dim, **kw)  # row T = bootstrap obs
        self.pre_tanh = torch.zeros(T, E, action_dim, **kw)
        self.actions = torch.zeros(T, E, action_dim, **kw)
        self.log_probs = torch.zeros(T, E, **kw)
        self.values = torch.zeros(T, E, **kw)
        self.rewards = torch.zeros(T, E, **kw)
        self.terminated = torch.zeros(T, E, device=device, dtype=torch.uint8)
        self.truncated = torch.zeros(T, E, device=device, dtype=torch.uint8)
        self.dones = torch.zeros(T, E, device=device, dtype=torch.uint8)
        self.ep_return = torch.zeros(T, E, **kw)
        self.ep_length = torch.zeros(T, E, device=device, dtype=torch.int32)
        self.noise = torch.zeros(T, E, action_dim, **kw)  # the rollout's sampling noise

    @property
    def n(self) -> int:
        return self.T * self.E

    def draw_noise(self, generator: Optional[torch.Generator] = None) -> None:
        """All T steps' standard normal sampling noise in one draw (one launch per rollout
        instead of one per step); step t acts with ``noise[t]``."""
        torch.randn(self.noise.shape, generator=generator, device=self.noise.device,
                    out=self.noise)

    def finish_dones(self) -> None:
        """dones = terminated | truncated for the whole rollout, once."""
        torch.bitwise_or(self.terminated, self.truncated, out=self.dones)


class _Learner:
    """Per-minibatch clipped-PPO step over a flattened device rollout, optionally graph-captured.

    Semantics per minibatch (ppo/agent.py:216-262): ratio = exp(logp - old); kl = mean(ratio - 1
    - log ratio); surrogate clipped at 1 +- eps; MSE value loss against returns; loss = pg +
    vc*vf - ec*entropy; zero grad, backward, [all-reduce mean], clip_grad_norm_, Adam step.
    Batch metrics land in a device buffer row per minibatch; nothing syncs with the host.
    """

    def __init__(self, agent: "PPOAgent", n: int, mb: int, n_steps: int, use_graph: bool,
                 group=None):
        self.agent = agent
        ac = agent.actor_critic
        dev = agent.device
        self.params = [p for p in ac.parameters()]
        numel = sum(p.numel() for p in self.params)
        self.flat_grad = torch.zeros(numel, device=dev, dtype=torch.float32)
        off = 0
        for p in self.params:
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.group = group
        self.world = 1 if group is None else torch.distributed.get_world_size(group)
        self.mb = mb
        self.n = n
        self.idx = torch.zeros(mb, dtype=torch.int64, device=dev)
        self.metrics = torch.zeros(max(1, n_steps), len(METRIC_KEYS), device=dev)
        self.row = torch.zeros((), dtype=torch.int64, device=dev)
        self.src: Dict[str, torch.Tensor] = {}
        self.use_graph = use_graph and dev.type == "cuda"
        self.g_fwd = self.g_opt = None

    def activate(self):
        """Point every parameter's .grad at this learner's flat buffer (another cached learner,
        or FusedPPO's flat gradient, may hold them); the same views, so captured graphs stay
        valid."""
        p0 = self.params[0]
        if p0.grad is None or p0.grad.data_ptr() != self.flat_grad.data_ptr():
            off = 0
            for p in self.params:
                p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
                off += p.numel()

    def bind(self, states, pre_tanh, old_logp, adv, ret):
        same = all(self.src.get(k) is v for k, v in (("s", states), ("z", pre_tanh),
                                                      ("lp", old_logp), ("a", adv), ("r", ret)))
        if not same:
            self.src = dict(s=states, z=pre_tanh, lp=old_logp, a=adv, r=ret)
            self.g_fwd = self.g_opt = None  # new storage -> recapture

    def _fwd_bwd(self):
        ag = self.agent
        s = self.src["s"].index_select(0, self.idx)
        z = self.src["z"].index_select(0, self.idx)
        old = self.src["lp"].index_select(0, self.idx)
        a = self.src["a"].index_select(0, self.idx)
        r = self.src["r"].index_select(0, self.idx)
        new_lp, values, ent = ag.actor_critic.evaluate(s, torch.tanh(z), z)
        log_ratio = new_lp - old
        ratios = torch.exp(log_ratio)
        surr1 = ratios * a
        surr2 = torch.clamp(ratios, 1 - ag.eps_clip, 1 + ag.eps_clip) * a
        actor_loss = -torch.min(surr1, surr2).mean()
        critic_loss = F.mse_loss(values.squeeze(-1), r)
        ent_b = ent.mean()
        loss = actor_loss + ag.value_coef * critic_loss - ag.entropy_coef * ent_b
        self.flat_grad.zero_()
        loss.backward()
        with torch.no_grad():
            kl = ((ratios - 1) - log_ratio).mean()
            clip = (torch.abs(ratios - 1) > ag.eps_clip).float().sum()  # / size on the host
            vals = torch.stack([actor_loss, critic_loss, ent_b, loss, clip, kl]).detach()
            self.metrics.index_copy_(0, self.row.view(1), vals.view(1, -1))

    def _opt(self):
        ag = self.agent
        nn.utils.clip_grad_norm_(self.params, ag.max_grad_norm, foreach=True)
        ag.optimizer.step()
        self.row.add_(1)

    def _allreduce(self):
        if self.group is not None:
            torch.distributed.all_reduce(self.flat_grad, group=self.group)
            self.flat_grad.div_(self.world)

    def _capture(self):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):  # warm-up builds autograd / optimizer state eagerly
            for _ in range(2):
                self._fwd_bwd()
                self._allreduce()
                self._opt()
        torch.cuda.current_stream().wait_stream(s)
        self.g_fwd, self.g_opt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with graph_capture(self.g_fwd):
            self._fwd_bwd()
        with graph_capture(self.g_opt):
            self._opt()

    def step(self, idx: torch.Tensor):
        self.idx.copy_(idx)
        if self.use_graph:
            if self.g_fwd is None:
                saved = [p.detach().clone() for p in self.params]
                opt_state = {k: {kk: (vv.clone() if torch.is_tensor(vv) else vv)
                                 for kk, vv in v.items()} for k, v in self.agent.optimizer.state.items()}
                row = self.row.clone()
                self._capture()
                with torch.no_grad():  # undo the warm-up steps
                    for p, v in zip(self.params, saved):
                        p.copy_(v)
                    for k, st in self.agent.optimizer.state.items():
                        for kk, vv in st.items():
                            if not torch.is_tensor(vv):
                                continue
                            if k in opt_state:
                                vv.copy_(opt_state[k][kk])
                            else:  # state created by the warm-up: back to a fresh Adam
                                vv.zero_()
                    self.row.copy_(row)
            self.g_fwd.replay()
            self._allreduce()
            self.g_opt.replay()
        else:
            self._fwd_bwd()
            self._allreduce()
            self._opt()


class _PendingMetrics:
    """An update's metrics dict whose device-to-host copy is in flight (non-blocking, pinned):
    result() waits for it, so a caller can enqueue the next rollout before reading them."""

    def __init__(self, logger, vals: torch.Tensor):
        self.logger = logger
        self._out = None
        if vals.is_cuda:
            self._host = torch.empty(vals.shape, dtype=vals.dtype, pin_memory=True)
            self._host.copy_(vals, non_blocking=True)
            self._event = torch.cuda.Event()
            self._event.record()
        else:
            self._host, self._event = vals, None

    def result(self) -> Dict[str, float]:
        if self._out is not None:
            return self._out
        if self._event is not None:
            self._event.synchronize()
        vals = self._host.tolist()
        m = dict(zip(METRIC_KEYS, vals[:-1]))
        out = {
            "loss": m["loss"],
            "policy_loss": m["policy_loss"],
            "value_loss": m["value_loss"],
            "entropy": m["entropy"],
            "clip_fraction": m["clip_fraction"],
            "approx_kl": m["approx_kl"],
            "explained_variance": vals[-1],
        }
        self.logger.info(
            "update_complete loss=%.4f policy_loss=%.4f value_loss=%.4f entropy=%.4f "
            "clip_frac=%.3f kl=%.5f explained_var=%.3f", out["loss"], out["policy_loss"],
            out["value_loss"], out["entropy"], out["clip_fraction"], out["approx_kl"],
            out["explained_variance"])
        self._out = out
        return out


class PPOAgent:
    def __init__(self, state_dim: int, action_dim: int, lr: float = 1e-4, gamma: float = 0.99,
                 lam: float = 0.95, eps_clip: float = 0.2, value_coef: float = 0.5,
                 entropy_coef: float = 0.005, max_grad_norm: float = 0.5, epochs: int = 6,
                 batch_size: int = 64, hidden_dim: int = 128,
                 logger: Optional[logging.Logger] = None,
                 device: torch.device = torch.device("cpu"),
                 num_minibatches: Optional[int] = None, use_graphs: bool = True,
                 process_group=None, seed: Optional[int] = None, backend: str = "auto"):
        self.device = torch.device(device)
        if backend not in ("auto", "hip", "torch"):
            raise ValueError(f"backend must be auto|hip|torch, got {backend!r}")
        # "hip": update_rollout runs the fused HIP minibatch step (hwy/ppo_native.py);
        # "torch": autograd + torch.optim.Adam (the reference arithmetic, also used by update())
        self.backend = backend
        self._fused = None
        self.actor_critic = ActorCritic(state_dim, action_dim, hidden_dim, device=self.device)
        self._dist = process_group
        if process_group is not None:  # identical initial weights on every rank
            for p in self.actor_critic.parameters():
                torch.distributed.broadcast(p.data, src=0, group=process_group)
        capturable = self.device.type == "cuda"
        self.optimizer = torch.optim.Adam(self.actor_critic.parameters(), lr=lr,
                                          capturable=capturable)
        self.gamma, self.lam, self.eps_clip = gamma, lam, eps_clip
        self.value_coef, self.entropy_coef = value_coef, entropy_coef
        self.max_grad_norm, self.epochs, self.batch_size = max_grad_norm, epochs, batch_size
        self.num_minibatches = num_minibatches
        self.use_graphs = use_graphs
        self.logger = logger or logging.getLogger(__name__)
        self.memory = PPOMemory(batch_size=batch_size, device=self.device)
        # torch-path learners, one per (rows, minibatch, steps, graph) geometry: a ragged
        # partition alternates between two sizes without reallocating
        self._learners: Dict[tuple, _Learner] = {}
        # which optimizer holds the current Adam state: "torch" (agent.optimizer) or "fused"
        # (FusedPPO's m / v / step); handed over whenever an update switches paths
        self._adam_owner = "torch"
        self._warned_ragged = False
        self.updates = 0  # completed update() / update_rollout() calls (evaluation memo key)
        # torch-path optimizer runs: a graph-replayed torch learner writes the parameters in
        # place without bumping their version counters, so the fused path's weight tile images
        # key their staleness on this count too (hwy/ppo_native.py)
        self._torch_param_writes = 0
        self.generator = None
        if self.device.type == "cuda":
            self.generator = torch.Generator(device=self.device)
            self.generator.manual_seed(int(seed) if seed is not None else torch.initial_seed() % (2**63))

    # ------------------------------------------------------------------ acting
    def select_action(self, state, deterministic: bool = False, out=None, noise=None):
        """Batched (2-D tensor) or single-state acting.  For a batch, `out` may name the four
        tensors (action, pre_tanh, log_prob, value) to write, e.g. a rollout buffer's rows, and
        `noise` a pre-drawn (B, action_dim) standard normal sample (RolloutBuffer.draw_noise)."""
        if isinstance(state, torch.Tensor) and state.dim() == 2:
            if self._act_fused_ok(state):
                from hwy.ppo_native import fused_act

                return fused_act(self, state, deterministic, self.generator, out=out, noise=noise)
            res = self.actor_critic.act(state, deterministic, generator=self.generator,
                                        noise=noise)
            if out is None:
                return res
            for dst, src in zip(out, res):
                dst.copy_(src.reshape(dst.shape))
            return tuple(out)
        return self.actor_critic.get_action(state, deterministic)

    def value(self, states: torch.Tensor) -> torch.Tensor:
        """V(s) for a batch, e.g. a rollout's bootstrap row: the value output of the fused act
        launch when acting is fused, else the torch forward."""
        if self._act_fused_ok(states):
            from hwy.ppo_native import fused_act

            return fused_act(self, states.contiguous(), True)[3]
        with torch.no_grad():
            return self.actor_critic.forward(states)[2].squeeze(-1)

    def _act_fused_ok(self, state: torch.Tensor) -> bool:
        """Batched acting runs through hwy_ppo_act (one launch) unless backend='torch'."""
        if self.backend == "torch" or not state.is_cuda:
            return False
        from hwy.ppo_native import act_supported

        H = self.actor_critic.shared[0].weight.shape[0]
        ok = act_supported(state.shape[1], H, self.actor_critic.log_std.numel())
        if not ok and self.backend == "hip":
            raise ValueError("backend='hip' acting needs action_dim 2, state_dim % 4 == 0 "
                             "(<= 256) and hidden_dim in {64,128,...,512}")
        return ok

    # ------------------------------------------------------------------ metrics
    def _finish_metrics(self, rows: torch.Tensor, sizes: List[int], values, returns,
                        deferred: bool = False):
        """Aggregate per-minibatch rows like ppo/agent.py:263-287 (epoch means, then the mean
        over epochs, in float64) plus explained variance (:272-280).  Computed on the rows'
        device with one host transfer at the end (the clip count becomes a fraction by dividing
        by each minibatch's size, as the reference's per-batch clip_frac).  ``deferred``: return
        a pending result whose host copy is still in flight (see _PendingMetrics)."""
        nb = len(sizes)
        r = torch.as_tensor(rows).to(torch.float64)[: self.epochs * nb].view(self.epochs, nb, -1)
        ci = METRIC_KEYS.index("clip_fraction")
        inv = torch.tensor([1.0 / s for s in sizes], dtype=torch.float64, device=r.device)
        r = torch.cat([r[..., :ci], r[..., ci:ci + 1] * inv.view(1, nb, 1), r[..., ci + 1:]], -1)
        means = r.mean(dim=1).mean(dim=0)  # epoch means, then over epochs
        with torch.no_grad():
            var_y = torch.var(returns)
            ev = torch.where(var_y > 0, 1 - torch.var(returns - values) / var_y,
                             torch.zeros_like(var_y)).to(torch.float64).to(means.device)
        pending = _PendingMetrics(self.logger, torch.cat([means, ev.view(1)]))
        return pending if deferred else pending.result()

    def _learner_for(self, n: int, mb: int, steps: int, graph: bool) -> _Learner:
        key = (n, mb, steps, graph)
        L = self._learners.get(key)
        if L is None:
            L = _Learner(self, n, mb, steps, graph, group=self._dist)
            self._learners[key] = L
        L.activate()
        return L

    def _adam_to(self, owner: str):
        """Hand the Adam state (moments, step count) to the optimizer about to step."""
        if owner == self._adam_owner:
            return
        F = self._fused
        if F is not None:
            if owner == "torch":
                F.export_torch_state()
            else:
                F._import_torch_state()
        self._adam_owner = owner

    def _run_epochs(self, states, pre_tanh, old_logp, adv, ret, batches: List[torch.Tensor]):
        self._adam_to("torch")
        self._torch_param_writes += 1  # retires every fused tile image (see __init__)
        n = states.shape[0]
        sizes = {int(b.numel()) for b in batches}
        mb = max(sizes)
        ragged = len(sizes) > 1
        steps = self.epochs * len(batches)
        if ragged:  # short last minibatch (reference's n % batch_size != 0): eager, exact sizes
            rows = []
            for _ in range(self.epochs):
                for b in batches:
                    L = self._learner_for(n, int(b.numel()), 1, False)
                    L.bind(states, pre_tanh, old_logp, adv, ret)
                    L.row.zero_()
                    L.step(b)
                    rows.append(L.metrics[0].clone())
            return torch.stack(rows)
        L = self._learner_for(n, mb, steps, self.use_graphs)
        L.bind(states, pre_tanh, old_logp, adv, ret)
        L.row.zero_()
        for _ in range(self.epochs):
            for b in batches:
                L.step(b)
        return L.metrics

    # ------------------------------------------------------------------ reference update
    def update(self, last_value: float = 0.0):
        """Clipped-PPO update over the list memory (ppo/agent.py:196-308)."""
        states, actions, pre_tanh, old_log_probs = self.memory.get_tensors()
        adv_np, ret_np = self.memory.compute_advantages(self.gamma, self.lam, last_value)
        advantages = torch.as_tensor(adv_np, device=self.device)
        returns = torch.as_tensor(ret_np, device=self.device)
        advantages = (advantages - advantages.mean()) / (advantages.std() + 1e-8)
        batches = [torch.as_tensor(b, device=self.device) for b in self.memory.get_batches()]
        rows = self._run_epochs(states, pre_tanh, old_log_probs, advantages, returns, batches)
        values = torch.as_tensor(np.asarray(self.memory.values, np.float32), device=self.device)
        out = self._finish_metrics(rows, [int(b.numel()) for b in batches], values,
                                   returns)
        self.memory.clear()
        self.updates += 1
        return out

    # ------------------------------------------------------------------ batched update
    def normalize_advantages(self, adv: torch.Tensor) -> torch.Tensor:
        """(adv - mean) / (unbiased std + 1e-8) over ALL ranks' samples (ppo/agent.py:204)."""
        if self._dist is None:
            return (adv - adv.mean()) / (adv.std() + 1e-8)
        a64 = adv.double()
        stats = torch.stack([torch.tensor(float(adv.numel()), device=adv.device, dtype=torch.float64),
                             a64.sum(), (a64 * a64).sum()])
        torch.distributed.all_reduce(stats, group=self._dist)
        n, s1, s2 = stats[0], stats[1], stats[2]
        mean = s1 / n
        var = (s2 - n * mean * mean) / (n - 1)
        return ((adv - mean.float()) / (var.clamp_min(0).sqrt().float() + 1e-8))

    def update_rollout(self, buf: RolloutBuffer, last_values: torch.Tensor,
                       perm: Optional[torch.Tensor] = None, return_metrics=True):
        """Batched clipped-PPO update on a device rollout (no host round trips until the end).
        return_metrics: True -> the metrics dict; "deferred" -> a pending result (metrics
        computed on the device, host copy in flight; .result() gives the dict); False -> the
        device rows only."""
        from hwy import ops

        T, E = buf.T, buf.E
        adv, ret = ops.gae(buf.rewards, buf.dones, buf.values, last_values, self.gamma, self.lam)
        n = T * E
        states = buf.states[:T].reshape(n, -1)
        pre_tanh = buf.pre_tanh.reshape(n, -1)
        old_lp = buf.log_probs.reshape(n)
        ret = ret.reshape(n)
        adv = self.normalize_advantages(adv.reshape(n))
        if perm is None:
            perm = torch.randperm(n, device=self.device, generator=self.generator)
        sizes = self.minibatch_sizes(n)
        mb, nmb = sizes[0], len(sizes)
        if len(set(sizes)) == 1 and self._fused_ok(mb):
            F = self._fused_for(mb, nmb, n)
            self._adam_to("fused")
            F_adv, F_ret, F_perm = self._static_bufs
            F_adv.copy_(adv)
            F_ret.copy_(ret)
            F_perm.copy_(perm)
            rows = F.run(states, pre_tanh, old_lp, F_adv, F_ret, F_perm)
        else:
            # one partition for all epochs (ppo/agent.py:205); a short last minibatch takes the
            # reference's ragged path (eager torch steps at the exact sizes)
            if len(set(sizes)) > 1 and not self._warned_ragged and self._fused_ok(mb):
                self._warned_ragged = True
                self.logger.warning(
                    f"update_rollout: {n} samples split into unequal minibatches {sorted(set(sizes))}"
                    " -- the fused HIP update needs equal sizes, so these updates run the eager "
                    "torch path (choose num_minibatches / batch_size dividing T x E)")
            starts = np.cumsum([0] + sizes)
            batches = [perm[int(starts[i]):int(starts[i + 1])] for i in range(nmb)]
            rows = self._run_epochs(states, pre_tanh, old_lp, adv, ret, batches)
        self.updates += 1
        if not return_metrics:
            return rows
        return self._finish_metrics(rows, sizes, buf.values.reshape(n), ret,
                                    deferred=return_metrics == "deferred")

    def minibatch_sizes(self, n: int) -> List[int]:
        """The minibatch partition of an n-sample update; every sample is used once per epoch.

        ``num_minibatches`` set: that many near-equal minibatches (the first n % nmb one row
        larger).  Otherwise the reference's get_batches partition (ppo/agent.py:140-146):
        ``batch_size`` rows each and a short last minibatch when batch_size does not divide n."""
        if self.num_minibatches:
            nmb = max(1, min(int(self.num_minibatches), n))
            q, r = divmod(n, nmb)
            sizes = [q + 1] * r + [q] * (nmb - r)
        else:
            bs = max(1, int(self.batch_size))
            sizes = [bs] * (n // bs) + ([n % bs] if n % bs else [])
        assert sum(sizes) == n, (sizes, n)
        return sizes

    # ------------------------------------------------------------------ fused HIP step
    def _fused_ok(self, mb: int) -> bool:
        if self.backend == "torch" or self.device.type != "cuda":
            return False
        sd = self.actor_critic.shared[0].weight
        H = sd.shape[0]
        ok = self.actor_critic.log_std.numel() == 2 and H % 64 == 0 and 64 <= H <= 512
        if not ok and self.backend == "hip":
            raise ValueError("backend='hip' needs action_dim 2 and hidden_dim in {64,128,...,512}")
        return ok

    def _fused_for(self, mb: int, nmb: int, n: int):
        from hwy.ppo_native import FusedPPO

        F = self._fused
        if F is None or F.mb != mb or F.nmb != nmb or F.metrics.shape[0] != self.epochs * nmb:
            if F is not None and self._adam_owner == "fused":
                F.export_torch_state()  # carry Adam's moments and step count to the new instance
            self._adam_owner = "torch"  # the new instance imports agent.optimizer's state
            F = FusedPPO(self, mb, nmb, group=self._dist, use_graphs=self.use_graphs)
            self._fused = F
            self._learners = {}
        bufs = getattr(self, "_static_bufs", None)
        if bufs is None or bufs[0].numel() != n:
            dev = self.device
            self._static_bufs = (torch.empty(n, device=dev), torch.empty(n, device=dev),
                                 torch.empty(n, device=dev, dtype=torch.int64))
        return F

    # ------------------------------------------------------------------ checkpoints
    def save(self, path: str):
        if self._fused is not None and self._adam_owner == "fused":
            self._fused.export_torch_state()
        torch.save({"model": self.actor_critic.state_dict(),
                    "optimizer": self.optimizer.state_dict()}, path)
        self.logger.info(f"model_saved path={path}")

    def load(self, path: str, load_optimizer: bool = True):
        ckpt = torch.load(path, map_location=self.device, weights_only=True)
        self.actor_critic.load_state_dict(ckpt["model"])
        if load_optimizer and "optimizer" in ckpt:
            self.optimizer.load_state_dict(ckpt["optimizer"])
            if self._fused is not None and self._adam_owner == "fused":
                self._fused._import_torch_state()
        self._learners = {}
        self.logger.info(f"model_loaded path={path}")
        return ckpt.get("config", {})
