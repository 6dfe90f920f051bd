"""Driver of the fused PPO minibatch step in libhwy.so (include/hwy_ppo.h).

``FusedPPO`` owns the flat parameter / gradient / Adam buffers of an ActorCritic (the module's
parameters are re-pointed into the flat buffer, so state_dict(), checkpoints and the torch
forward used for acting see the same storage) and runs one update's minibatch steps:

  * single GPU: one HIP graph per epoch (minibatch i uses perm[i*mb:(i+1)*mb] of a static
    permutation buffer; the same partition is replayed for every epoch, ppo/agent.py:205);
  * with a process group: per minibatch, graph(forward+backward) -> RCCL all-reduce of the flat
    gradient (mean) -> graph(clip + Adam).
"""

from __future__ import annotations

import ctypes
import gc
import os
from typing import List, Optional

import torch

from utils.graphs import capture as graph_capture

from .native import check, lib, stream_ptr

_PARAM_ORDER = ("shared.0.weight", "shared.0.bias", "shared.2.weight", "shared.2.bias",
                "actor_mean.0.weight", "actor_mean.0.bias", "actor_mean.2.weight",
                "actor_mean.2.bias", "log_std", "critic.0.weight", "critic.0.bias",
                "critic.2.weight", "critic.2.bias")


class PpoDims(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int32), ("S", ctypes.c_int32), ("H", ctypes.c_int32),
                ("A", ctypes.c_int32)]


class PpoArgs(ctypes.Structure):
    _fields_ = [
        ("dims", PpoDims),
        ("states", ctypes.c_void_p), ("pre_tanh", ctypes.c_void_p), ("old_logp", ctypes.c_void_p),
        ("adv", ctypes.c_void_p), ("ret", ctypes.c_void_p), ("idx", ctypes.c_void_p),
        ("params", ctypes.c_void_p), ("grads", ctypes.c_void_p), ("adam_m", ctypes.c_void_p),
        ("adam_v", ctypes.c_void_p), ("counters", ctypes.c_void_p), ("metrics", ctypes.c_void_p),
        ("workspace", ctypes.c_void_p),
        ("eps_clip", ctypes.c_float), ("value_coef", ctypes.c_float),
        ("entropy_coef", ctypes.c_float), ("max_grad_norm", ctypes.c_float),
        ("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float),
        ("adam_eps", ctypes.c_float), ("grads_modified", ctypes.c_int32),
    ]


class PpoActArgs(ctypes.Structure):
    _fields_ = [
        ("dims", PpoDims),
        ("states", ctypes.c_void_p), ("params", ctypes.c_void_p), ("noise", ctypes.c_void_p),
        ("action", ctypes.c_void_p), ("pre_tanh", ctypes.c_void_p), ("logp", ctypes.c_void_p),
        ("value", ctypes.c_void_p), ("tiles", ctypes.c_void_p),
    ]


def _bind(L):
    if getattr(L, "_ppo_bound", False):
        return L
    L.hwy_ppo_param_layout.argtypes = [ctypes.POINTER(PpoDims), ctypes.c_void_p, ctypes.c_void_p]
    L.hwy_ppo_param_layout.restype = ctypes.c_int
    L.hwy_ppo_workspace_bytes.argtypes = [ctypes.POINTER(PpoDims)]
    L.hwy_ppo_workspace_bytes.restype = ctypes.c_int64
    L.hwy_ppo_forward_backward.argtypes = [ctypes.POINTER(PpoArgs), ctypes.c_void_p]
    L.hwy_ppo_forward_backward.restype = ctypes.c_int
    L.hwy_ppo_optimizer.argtypes = [ctypes.POINTER(PpoArgs), ctypes.c_void_p]
    L.hwy_ppo_optimizer.restype = ctypes.c_int
    L.hwy_ppo_sync_params.argtypes = [ctypes.POINTER(PpoArgs), ctypes.c_void_p]
    L.hwy_ppo_sync_params.restype = ctypes.c_int
    L.hwy_ppo_act.argtypes = [ctypes.POINTER(PpoActArgs), ctypes.c_void_p]
    L.hwy_ppo_act.restype = ctypes.c_int
    L.hwy_ppo_time_kernels.argtypes = [ctypes.POINTER(PpoArgs), ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_void_p]
    L.hwy_ppo_time_kernels.restype = ctypes.c_int
    L.hwy_ppo_tile_image_offset.argtypes = [ctypes.POINTER(PpoDims)]
    L.hwy_ppo_tile_image_offset.restype = ctypes.c_int64
    # grouped learners (include/hwy_ppo.h)
    L.hwy_ppo_group_table_bytes.argtypes = [ctypes.POINTER(PpoDims), ctypes.c_int]
    L.hwy_ppo_group_table_bytes.restype = ctypes.c_int64
    L.hwy_ppo_group_act_table_bytes.argtypes = [ctypes.c_int]
    L.hwy_ppo_group_act_table_bytes.restype = ctypes.c_int64
    L.hwy_ppo_group_act_prepare.argtypes = [ctypes.POINTER(PpoActArgs), ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p]
    L.hwy_ppo_group_act_prepare.restype = ctypes.c_int
    L.hwy_ppo_group_act.argtypes = [ctypes.POINTER(PpoDims), ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p]
    L.hwy_ppo_group_act.restype = ctypes.c_int
    L._ppo_bound = True
    return L


def param_layout(S: int, H: int, B: int = 64):
    L = _bind(lib())
    d = PpoDims(B, S, H, 2)
    offs = (ctypes.c_int64 * 13)()
    n = ctypes.c_int64()
    if L.hwy_ppo_param_layout(ctypes.byref(d), offs, ctypes.byref(n)) != 0:
        raise ValueError(f"fused PPO supports action_dim 2 and hidden_dim a multiple of 64 "
                         f"(<= 512); got S={S} H={H}")
    return list(offs), int(n.value)


def flat_params(agent):
    """The ActorCritic's parameters (and gradients) as views of one flat fp32 buffer in
    hwy_ppo_param_layout order, created once per agent and shared by FusedPPO and fused_act."""
    cached = getattr(agent, "_flat", None)
    ac = agent.actor_critic
    # fast path (every acting call lands here): the same module objects still hold the same
    # parameters, still viewing the flat buffer -- checked through the modules' own dicts, not
    # named_parameters(), whose module walk cost ~50 us per call
    guard = getattr(agent, "_flat_guard", None)
    if cached is not None and guard is not None and guard[0] is ac:
        ok = True
        for steps, p, ptr in guard[1]:
            for d, k, obj in steps:
                if d.get(k) is not obj:
                    ok = False
                    break
            if not ok or p.data.data_ptr() != ptr:
                ok = False
                break
        if ok:
            return cached
    named = dict(ac.named_parameters())
    if cached is not None and all(named[n].data.data_ptr() == cached[0][o:].data_ptr()
                                  for n, o in zip(_PARAM_ORDER, cached[2])):
        agent._flat_guard = _flat_guard(ac, cached[0], cached[2])
        return cached
    if set(named.keys()) != set(_PARAM_ORDER):
        raise ValueError("unexpected ActorCritic parameter layout for the fused step")
    S = named["shared.0.weight"].shape[1]
    H = named["shared.0.weight"].shape[0]
    if named["log_std"].numel() != 2:
        raise ValueError("fused PPO step needs action_dim == 2")
    offs, numel = param_layout(S, H)
    dev = named["log_std"].device
    flat = torch.empty(numel, device=dev, dtype=torch.float32)
    grads = torch.zeros(numel, device=dev, dtype=torch.float32)
    params: List[torch.nn.Parameter] = []
    with torch.no_grad():
        for name, off in zip(_PARAM_ORDER, offs):
            p = named[name]
            n = p.numel()
            flat[off:off + n].copy_(p.detach().reshape(-1))
            p.data = flat[off:off + n].view_as(p)
            p.grad = grads[off:off + n].view_as(p)
            params.append(p)
    agent._flat = (flat, grads, offs, params)
    agent._flat_guard = _flat_guard(ac, flat, offs)
    agent._learners = {}  # a torch-graph learner captured the old storage
    return agent._flat


def _flat_guard(ac, flat: torch.Tensor, offs) -> tuple:
    """flat_params' fast-path check: per parameter the chain of (module dict, key, object) from
    the ActorCritic down to it, the Parameter, and the flat-buffer address it must view."""
    out = []
    for name, off in zip(_PARAM_ORDER, offs):
        parts = name.split(".")
        steps, mod = [], ac
        for part in parts[:-1]:
            child = mod._modules[part]
            steps.append((mod._modules, part, child))
            mod = child
        p = mod._parameters[parts[-1]]
        steps.append((mod._parameters, parts[-1], p))
        out.append((tuple(steps), p, flat[off:].data_ptr()))
    return (ac, tuple(out))


def _param_versions(agent, flat: torch.Tensor, params) -> tuple:
    """What a weight tile image is in step with: in-place writes through a parameter
    (load_state_dict, an eager torch optimizer step) bump that parameter's version counter, writes
    through the flat buffer bump the buffer's, and a graph-replayed torch learner, which writes in
    place without bumping either, counts in agent._torch_param_writes."""
    return ((getattr(agent, "_torch_param_writes", 0), flat._version)
            + tuple(p._version for p in params))


# hidden width at which hwy_ppo_act runs ppo_act_c, the forward + head of the minibatch step's
# compact row kernel, from a weight tile image (ppo_kernels.hip: hwy_ppo_act)
_ACT_C_HIDDEN = 256


class _TileImage:
    """A weight tile image (hwy_ppo_sync_params) for acting when no FusedPPO keeps one in step
    with the parameters: a fresh agent, or a checkpoint loaded before the first fused update.
    At H = 256 acting then always runs ppo_act_c, whose bits are the minibatch step's, instead of
    ppo_act on the params rows (equal only to fp32 rounding)."""

    def __init__(self, agent, flat: torch.Tensor, S: int, H: int):
        L = _bind(lib())
        self.L, self.flat, self.S = L, flat, S
        self.agent = agent
        self.params = flat_params(agent)[3]
        self.dims = PpoDims(64, S, H, 2)
        ws = L.hwy_ppo_workspace_bytes(ctypes.byref(self.dims))
        off = L.hwy_ppo_tile_image_offset(ctypes.byref(self.dims))
        if ws < 0 or off < 0:
            raise ValueError("unsupported fused PPO dims for a tile image")
        self.workspace = torch.zeros(int(ws), device=flat.device, dtype=torch.uint8)
        self.off = int(off)
        self.version = None

    def _versions(self):
        return _param_versions(self.agent, self.flat, self.params)

    def current(self) -> int:
        if self.version != self._versions():
            a = PpoArgs()
            a.dims = self.dims
            a.params, a.workspace = self.flat.data_ptr(), self.workspace.data_ptr()
            check(self.L.hwy_ppo_sync_params(ctypes.byref(a), stream_ptr()), "hwy_ppo_sync_params")
            self.version = self._versions()
        return self.workspace.data_ptr() + self.off


def _act_tiles(agent, flat: torch.Tensor, S: int, H: int) -> Optional[int]:
    """A tile image in step with `flat`: the agent's FusedPPO's, rebuilt from the params when a
    torch-side write retired it, else an acting-only one (_TileImage)."""
    F = getattr(agent, "_fused", None)
    if F is not None and F.flat is flat and F._tile_off is not None:
        F.refresh_tiles()
        return F.current_tiles(flat)
    T = getattr(agent, "_act_tile_image", None)
    if T is None or T.flat is not flat or T.S != S:
        T = agent._act_tile_image = _TileImage(agent, flat, S, H)
    return T.current()


def act_supported(S: int, H: int, A: int) -> bool:
    return A == 2 and S % 4 == 0 and S <= 256 and H % 64 == 0 and 64 <= H <= 512


def act_tiles(agent, flat: torch.Tensor, S: int, H: int) -> Optional[int]:
    """The weight tile image fused_act streams for this agent (None: the params rows): its
    FusedPPO's when in step, else at H = 256 an acting-only image (_act_tiles)."""
    F = getattr(agent, "_fused", None)
    t = F.current_tiles(flat) if F is not None else None
    if t is None and H == _ACT_C_HIDDEN:
        t = _act_tiles(agent, flat, S, H)
    return t


def fused_act(agent, states: torch.Tensor, deterministic: bool = False,
              generator: Optional[torch.Generator] = None, out=None,
              noise: Optional[torch.Tensor] = None):
    """ActorCritic.act (ppo/agent.py:86-95) through hwy_ppo_act: one launch for the forward,
    the Normal sample (noise drawn from `generator` exactly as act() draws it), tanh and the
    squashed log-prob.  Returns (action, pre_tanh, log_prob, value); `out` = four contiguous
    float32 device tensors of shapes (B, 2), (B, 2), (B,), (B,) to write them into instead
    (e.g. the rollout buffer rows of this step); `noise` = a pre-drawn contiguous float32
    (B, 2) standard normal sample to use instead of drawing one."""
    flat = flat_params(agent)[0]
    B, S = states.shape
    H = agent.actor_critic.shared[0].weight.shape[0]
    dev = states.device
    states = states.contiguous()
    if deterministic:
        noise = None
    elif noise is None:
        noise = torch.randn((B, 2), device=dev, dtype=states.dtype, generator=generator)
    elif (tuple(noise.shape) != (B, 2) or noise.dtype != torch.float32 or noise.device != dev
          or not noise.is_contiguous()):
        raise ValueError(f"fused_act noise must be contiguous float32 {(B, 2)} on {dev}")
    if out is None:
        action = torch.empty(B, 2, device=dev)
        pre = torch.empty(B, 2, device=dev)
        logp = torch.empty(B, device=dev)
        value = torch.empty(B, device=dev)
    else:
        action, pre, logp, value = out
        for t, shp in zip(out, ((B, 2), (B, 2), (B,), (B,))):
            if (tuple(t.shape) != shp or t.dtype != torch.float32 or t.device != dev
                    or not t.is_contiguous()):
                raise ValueError(f"fused_act out tensor must be contiguous float32 {shp} on {dev}")
    a = PpoActArgs()
    a.dims = PpoDims(B, S, H, 2)
    a.states, a.params = states.data_ptr(), flat.data_ptr()
    a.noise = None if noise is None else noise.data_ptr()
    a.action, a.pre_tanh, a.logp, a.value = (action.data_ptr(), pre.data_ptr(), logp.data_ptr(),
                                             value.data_ptr())
    a.tiles = act_tiles(agent, flat, S, H)
    check(_bind(lib()).hwy_ppo_act(ctypes.byref(a), stream_ptr()), "hwy_ppo_act")
    return action, pre, logp, value


class FusedPPO:
    def __init__(self, agent, mb: int, nmb: int, group=None, use_graphs: bool = True):
        ac = agent.actor_critic
        self.agent = agent
        dev = agent.device
        named = dict(ac.named_parameters())
        if set(named.keys()) != set(_PARAM_ORDER):
            raise ValueError("unexpected ActorCritic parameter layout for the fused step")
        S = named["shared.0.weight"].shape[1]
        H = named["shared.0.weight"].shape[0]
        if named["log_std"].numel() != 2:
            raise ValueError("fused PPO step needs action_dim == 2")
        self.S, self.H, self.mb, self.nmb = S, H, mb, nmb
        L = _bind(lib())
        self.L = L
        self.dims = PpoDims(mb, S, H, 2)
        ws = L.hwy_ppo_workspace_bytes(ctypes.byref(self.dims))
        if ws < 0:
            raise ValueError("unsupported fused PPO dims")
        self.flat, self.grads, self.offs, self.params = flat_params(agent)
        numel = self.flat.numel()
        self.m = torch.zeros(numel, device=dev, dtype=torch.float32)
        self.v = torch.zeros(numel, device=dev, dtype=torch.float32)
        self.workspace = torch.zeros(int(ws), device=dev, dtype=torch.uint8)
        self.counters = torch.zeros(2, device=dev, dtype=torch.int32)
        self.metrics = torch.zeros(max(1, agent.epochs * nmb), 6, device=dev)
        self.group = group
        self.world = 1 if group is None else torch.distributed.get_world_size(group)
        self._rccl = group is not None and torch.distributed.get_backend(group) == "nccl"
        self._avg_op = self._rccl
        # RCCL collectives are captured into the epoch graph with the kernels (one replay per
        # epoch, as on one GPU); HWY_GRAPH_COLLECTIVES=0 keeps them between per-step graphs
        self.capture_collectives = self._rccl and os.environ.get("HWY_GRAPH_COLLECTIVES", "1") != "0"
        self._captured_collectives = False
        self.use_graphs = use_graphs
        self._import_torch_state()
        self._graphs = None
        self._bound_key = None
        # when a list: (start, end) HIP events on the launch stream around every epoch's
        # minibatch steps are appended to it (bench.py's live timing of the update)
        self.epoch_events: Optional[list] = None
        off = L.hwy_ppo_tile_image_offset(ctypes.byref(self.dims))
        self._tile_off = int(off) if off >= 0 else None
        self._tiles_version = None  # flat._version when the tile image was last made current

    # -------------------------------------------------------------- optimizer state <-> torch
    def _import_torch_state(self):
        opt = self.agent.optimizer
        st0 = opt.state.get(self.params[0])
        if not st0:
            return
        with torch.no_grad():
            for p, off in zip(self.params, self.offs):
                st = opt.state[p]
                n = p.numel()
                self.m[off:off + n].copy_(st["exp_avg"].reshape(-1))
                self.v[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
            self.counters[0] = int(float(st0["step"]))

    def export_torch_state(self):
        """Write the fused Adam state into agent.optimizer (torch.optim.Adam layout)."""
        opt = self.agent.optimizer
        t = int(self.counters[0].item())
        if t == 0:
            return
        with torch.no_grad():
            for p, off in zip(self.params, self.offs):
                n = p.numel()
                m, v = self.m[off:off + n].view_as(p), self.v[off:off + n].view_as(p)
                st = opt.state.get(p)
                if st and all(k in st for k in ("step", "exp_avg", "exp_avg_sq")) and \
                        st["exp_avg"].shape == p.shape:
                    # in place: a captured torch learner's graph still points at these tensors
                    st["exp_avg"].copy_(m)
                    st["exp_avg_sq"].copy_(v)
                    st["step"].fill_(float(t))
                    continue
                opt.state[p] = {
                    "step": torch.tensor(float(t), device=p.device if opt.defaults.get("capturable") else "cpu"),
                    "exp_avg": m.clone(),
                    "exp_avg_sq": v.clone(),
                }

    # -------------------------------------------------------------- steps
    def _args(self, states, pre_tanh, old_lp, adv, ret, idx_ptr: int) -> PpoArgs:
        ag = self.agent
        a = PpoArgs()
        a.dims = self.dims
        a.states, a.pre_tanh, a.old_logp = states.data_ptr(), pre_tanh.data_ptr(), old_lp.data_ptr()
        a.adv, a.ret, a.idx = adv.data_ptr(), ret.data_ptr(), idx_ptr
        a.params, a.grads = self.flat.data_ptr(), self.grads.data_ptr()
        a.adam_m, a.adam_v = self.m.data_ptr(), self.v.data_ptr()
        a.counters, a.metrics = self.counters.data_ptr(), self.metrics.data_ptr()
        a.workspace = self.workspace.data_ptr()
        a.eps_clip, a.value_coef, a.entropy_coef = ag.eps_clip, ag.value_coef, ag.entropy_coef
        a.max_grad_norm = ag.max_grad_norm
        g = ag.optimizer.param_groups[0]
        a.lr, (a.beta1, a.beta2), a.adam_eps = g["lr"], g["betas"], g["eps"]
        a.grads_modified = 1 if self.group is not None else 0
        return a

    def _scalar_key(self):
        ag = self.agent
        g = ag.optimizer.param_groups[0]
        return (float(ag.eps_clip), float(ag.value_coef), float(ag.entropy_coef),
                float(ag.max_grad_norm), float(g["lr"]), tuple(map(float, g["betas"])),
                float(g["eps"]))

    def _fwd_bwd(self, a):
        check(self.L.hwy_ppo_forward_backward(ctypes.byref(a), stream_ptr()), "hwy_ppo_forward_backward")

    def _opt(self, a):
        check(self.L.hwy_ppo_optimizer(ctypes.byref(a), stream_ptr()), "hwy_ppo_optimizer")

    def sync_params(self, a):
        """Rebuild the workspace's weight tile image from the flat params (hwy_ppo_sync_params);
        needed before a step whenever params changed outside hwy_ppo_optimizer."""
        check(self.L.hwy_ppo_sync_params(ctypes.byref(a), stream_ptr()), "hwy_ppo_sync_params")

    def refresh_tiles(self):
        """Rebuild the tile image from the flat params if a torch-side write retired it."""
        if self._tile_off is None or self._tiles_version == self._param_versions():
            return
        a = PpoArgs()
        a.dims = self.dims
        a.params, a.workspace = self.flat.data_ptr(), self.workspace.data_ptr()
        self.sync_params(a)
        self._tiles_version = self._param_versions()

    def current_tiles(self, flat: torch.Tensor) -> Optional[int]:
        """Device address of the weight tile image when it is in step with `flat` (it is after
        run(): hwy_ppo_optimizer rewrites it with the weights; any torch-side write to the
        parameters since -- load_state_dict, a torch optimizer step -- bumps a version counter
        and the caller reads params instead), else None."""
        if (self._tile_off is None or flat is not self.flat
                or self._tiles_version != self._param_versions()):
            return None
        return self.workspace.data_ptr() + self._tile_off

    def _param_versions(self):
        return _param_versions(self.agent, self.flat, self.params)

    def _allreduce(self):
        if self._avg_op:  # RCCL averages in the collective (no extra division kernel)
            try:
                torch.distributed.all_reduce(self.grads, op=torch.distributed.ReduceOp.AVG,
                                             group=self.group)
                return
            except RuntimeError:  # a collective library without ncclAvg: sum, then divide
                self._avg_op = False
        torch.distributed.all_reduce(self.grads, group=self.group)
        self.grads.div_(self.world)

    def run(self, states, pre_tanh, old_lp, adv, ret, perm: torch.Tensor) -> torch.Tensor:
        """All epochs of one update; returns the [epochs*nmb, 6] metrics rows (device)."""
        mb, nmb, epochs = self.mb, self.nmb, self.agent.epochs
        # Adam's state moves here if the agent's torch optimizer stepped last (ppo/agent.py);
        # an instance not (yet) registered as agent._fused takes the state over the same way
        ag = self.agent
        if hasattr(ag, "_adam_to") and getattr(ag, "_fused", None) in (None, self):
            # an unregistered instance registers as it takes the Adam state over, so the agent
            # can export it back (save(), a torch-path update) instead of using stale state
            ag._fused = self
            ag._adam_to("fused")
        # the captured graphs bake in the buffer addresses and the scalar hyper-parameters of
        # PpoArgs: a change to either (an lr schedule, agent.eps_clip, ...) forces a recapture
        key = (states.data_ptr(), pre_tanh.data_ptr(), old_lp.data_ptr(), adv.data_ptr(),
               ret.data_ptr(), perm.data_ptr()) + self._scalar_key()
        args = [self._args(states, pre_tanh, old_lp, adv, ret, perm.data_ptr() + i * mb * 8)
                for i in range(nmb)]
        self._last_args = args
        # the tensors behind args' raw addresses stay referenced while the args are kept
        # (time_kernels replays them later)
        self._last_inputs = (states, pre_tanh, old_lp, adv, ret, perm)
        self.counters[1].zero_()
        # the weight tile image the row kernel streams: params may have been written since the
        # last update (checkpoint load, torch optimizer); hwy_ppo_optimizer keeps it in step
        self.sync_params(args[0])
        if not self.use_graphs:
            for _ in range(epochs):
                ev = self._epoch_event()
                for a in args:
                    self._fwd_bwd(a)
                    if self.group is not None:
                        self._allreduce()
                    self._opt(a)
                self._epoch_event(ev)
            self._tiles_version = self._param_versions()
            return self.metrics
        if self._graphs is None or self._bound_key != key:
            self._capture(args)
            self._bound_key = key
        for _ in range(epochs):
            ev = self._epoch_event()
            if self.group is None or self._captured_collectives:
                self._graphs[0].replay()
            else:
                for gf, go in self._graphs:
                    gf.replay()
                    self._allreduce()
                    go.replay()
            self._epoch_event(ev)
        self._tiles_version = self._param_versions()
        return self.metrics

    KERNELS = ("ppo_rows", "ppo_wgrad", "ppo_wsum", "ppo_adam")

    def time_kernels(self, reps: int = 16) -> Optional[dict]:
        """Average microseconds per launch of each kernel of the minibatch step (ppo_rows,
        ppo_wgrad, ppo_wsum, ppo_adam) on the last update's first minibatch, each as a HIP graph
        of `reps` back-to-back launches (hwy_ppo_time_kernels), and of an empty kernel
        (`launch_floor`: the per-launch cost a kernel-trace duration leaves out).  A measurement
        aid for bench.py, run after its timed region.  The training state is left as it was
        (ADVICE r5): the repeated Adam launches step the weights, moments and tile image with one
        gradient, so params, Adam moments, counters and metrics are snapshotted before and put
        back after, and the tile image is rebuilt from the restored params.  None before the
        first run()."""
        args = getattr(self, "_last_args", None)
        if not args:
            return None
        # the last run's inputs are held with its args, so the addresses are still live
        a = PpoArgs.from_buffer_copy(args[0])
        a.grads_modified = 0  # this rank's own kernels only (no all-reduce between them)
        saved = [t.clone() for t in (self.flat, self.m, self.v, self.counters, self.metrics)]
        self.counters[1].zero_()
        us = (ctypes.c_float * 5)()
        check(self.L.hwy_ppo_time_kernels(ctypes.byref(a), stream_ptr(), max(1, int(reps)), us),
              "hwy_ppo_time_kernels")
        with torch.no_grad():
            for dst, src in zip((self.flat, self.m, self.v, self.counters, self.metrics), saved):
                dst.copy_(src)
        self.grads.zero_()
        self.sync_params(a)
        self._tiles_version = self._param_versions()
        return dict(zip(self.KERNELS + ("launch_floor",), (float(u) for u in us)))

    def release_graphs(self) -> None:
        """Drop the captured epoch / step graphs now (after the stream has drained).  Call it
        before tearing down the process group an RCCL-captured graph was built on: a graph whose
        collective outlives its communicator aborts in its destructor ("operation not permitted
        when stream is capturing"), and a graph in a reference cycle (agent <-> FusedPPO) is
        otherwise freed at an arbitrary later point."""
        torch.cuda.synchronize()
        self._graphs = None
        self._bound_key = None
        self._captured_collectives = False
        gc.collect()

    def _epoch_event(self, start=None):
        if self.epoch_events is None:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        if start is not None:
            self.epoch_events.append((start, e))
        return e

    def _capture(self, args):
        self._keep_args = args
        if self.capture_collectives and self._capture_with_collectives(args):
            return
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        graphs = []
        with torch.cuda.stream(s):
            if self.group is None:
                g = torch.cuda.CUDAGraph()
                with graph_capture(g, stream=s):
                    for a in args:
                        self._fwd_bwd(a)
                        self._opt(a)
                graphs.append(g)
            else:
                gc.collect()
                for a in args:
                    gf, go = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                    with graph_capture(gf, stream=s, collect=False):
                        self._fwd_bwd(a)
                    with graph_capture(go, stream=s, collect=False):
                        self._opt(a)
                    graphs.append((gf, go))
        torch.cuda.current_stream().wait_stream(s)
        self._graphs = graphs
        self._captured_collectives = False

    def _capture_with_collectives(self, args) -> bool:
        """One graph per epoch holding every step's forward/backward, the RCCL gradient
        all-reduce and the optimizer (the communicator is warmed up, and the AVG op probed,
        outside the capture).  False when the capture is refused: the caller falls back to
        per-step graphs with the all-reduce between them."""
        self._allreduce()  # communicator set-up + AVG support, before any capture
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.stream(s):
                # thread_local: the process group's watchdog thread may query events meanwhile
                with graph_capture(g, stream=s, capture_error_mode="thread_local"):
                    for a in args:
                        self._fwd_bwd(a)
                        self._allreduce()
                        self._opt(a)
        except RuntimeError:
            torch.cuda.synchronize()
            self.capture_collectives = False
            return False
        torch.cuda.current_stream().wait_stream(s)
        self._graphs = [g]
        self._captured_collectives = True
        return True


# ------------------------------------------------------------------ grouped learners
class PpoGroupPlan(ctypes.Structure):
    _fields_ = [("G", ctypes.c_int32), ("B", ctypes.c_int32), ("H", ctypes.c_int32),
                ("grid_rows", ctypes.c_int32), ("grid_wgrad", ctypes.c_int32),
                ("grid_wsum", ctypes.c_int32), ("grid_adam", ctypes.c_int32)]


def _bind_group(L):
    if getattr(L, "_grp_bound", False):
        return L
    L.hwy_ppo_group_prepare.argtypes = [ctypes.POINTER(PpoArgs), ctypes.c_int, ctypes.c_void_p,
                                        ctypes.POINTER(PpoGroupPlan), ctypes.c_void_p]
    L.hwy_ppo_group_prepare.restype = ctypes.c_int
    L.hwy_ppo_group_step.argtypes = [ctypes.POINTER(PpoGroupPlan), ctypes.c_void_p,
                                     ctypes.c_void_p]
    L.hwy_ppo_group_step.restype = ctypes.c_int
    L._grp_bound = True
    return L


class GroupAct:
    """ActorCritic.act for G agents (same hidden width and rows per agent; state dims may
    differ) in ONE launch (hwy_ppo_group_act): agent g acts on its own B rows and writes its own
    output rows, each bit for bit what fused_act(agent g, its rows) writes.  The kernel arguments
    live in a device table prepared once per (buffers, weights) key, so the launch is
    graph-capturable."""

    def __init__(self, agents, B: int):
        self.agents = list(agents)
        self.G, self.B = len(self.agents), int(B)
        self.L = _bind(lib())
        self.S = [ag.actor_critic.shared[0].weight.shape[1] for ag in self.agents]
        self.H = self.agents[0].actor_critic.shared[0].weight.shape[0]
        if any(ag.actor_critic.shared[0].weight.shape[0] != self.H for ag in self.agents):
            raise ValueError("grouped acting needs one hidden width")
        self.dims = PpoDims(self.B, self.S[0], self.H, 2)
        nb = self.L.hwy_ppo_group_act_table_bytes(self.G)
        self.dev = self.agents[0].device
        self._tables = {}
        self._nb = int(nb)

    def tiles(self):
        out = []
        for ag, S in zip(self.agents, self.S):
            flat = flat_params(ag)[0]
            out.append(act_tiles(ag, flat, S, self.H))
        return out

    def table(self, rows, tiles) -> torch.Tensor:
        """The device argument table for these row addresses (cached by them): rows[g] =
        (states, noise or None, action, pre_tanh, logp, value) device addresses of agent g."""
        key = (tuple(rows), tuple(tiles), tuple(flat_params(ag)[0].data_ptr() for ag in self.agents))
        t = self._tables.get(key)
        if t is not None:
            return t
        arr = (PpoActArgs * self.G)()
        for g, (ag, tl, r, S) in enumerate(zip(self.agents, tiles, rows, self.S)):
            a = arr[g]
            a.dims = PpoDims(self.B, S, self.H, 2)
            a.states, a.noise, a.action, a.pre_tanh, a.logp, a.value = r
            a.params = flat_params(ag)[0].data_ptr()
            a.tiles = tl
        t = torch.empty(self._nb, dtype=torch.uint8, device=self.dev)
        check(self.L.hwy_ppo_group_act_prepare(arr, self.G, t.data_ptr(), stream_ptr()),
              "hwy_ppo_group_act_prepare")
        self._tables[key] = t
        return t

    def rows_of(self, states, out, noise=None, first: int = 0, count: Optional[int] = None):
        """Row addresses of agents first..first+count acting on consecutive B-row blocks of one
        buffer set: states [count*B, S], out = (action [.,2], pre_tanh [.,2], logp [.], value [.]),
        noise [count*B, 2] or None."""
        count = self.G - first if count is None else count
        action, pre, logp, value = out
        B, S = self.B, self.S[first]
        rows = []
        for g in range(count):
            rows.append((states.data_ptr() + g * B * S * 4,
                         None if noise is None else noise.data_ptr() + g * B * 2 * 4,
                         action.data_ptr() + g * B * 2 * 4, pre.data_ptr() + g * B * 2 * 4,
                         logp.data_ptr() + g * B * 4, value.data_ptr() + g * B * 4))
        return rows

    def launch(self, rows, tiles=None):
        tiles = self.tiles() if tiles is None else tiles
        t = self.table(rows, tiles)
        check(self.L.hwy_ppo_group_act(ctypes.byref(self.dims), self.G,
                                       int(tiles[0] is not None), t.data_ptr(), stream_ptr()),
              "hwy_ppo_group_act")

    def __call__(self, states, out, noise=None, tiles=None):
        """All G agents on consecutive B-row blocks of one buffer set (see rows_of)."""
        self.launch(self.rows_of(states, out, noise), tiles)


class GroupStep:
    """One minibatch step of G FusedPPO learners (same rows and hidden width; state dims may
    differ) in four launches (hwy_ppo_group_step): learner g's arguments are its own
    FusedPPO._args, so each learner steps bit for bit as its solo run() would.  One device table
    (and plan) per minibatch index."""

    def __init__(self, fused):
        self.fused = list(fused)
        self.G = len(self.fused)
        F0 = self.fused[0]
        self.L = _bind_group(F0.L)
        if any(F.mb != F0.mb or F.H != F0.H for F in self.fused):
            raise ValueError("grouped PPO step: the learners share minibatch rows and hidden width")
        nb = self.L.hwy_ppo_group_table_bytes(ctypes.byref(F0.dims), self.G)
        if nb < 0:
            raise ValueError(f"grouped PPO step: unsupported dims B={F0.mb} S={F0.S} H={F0.H} "
                             "(16-row tiles: minibatches below 8,192 rows)")
        self._nb = int(nb)
        self.tables: List[torch.Tensor] = []
        self.plans: List[PpoGroupPlan] = []

    def prepare(self, per_learner_args) -> None:
        """per_learner_args[g][i]: learner g's PpoArgs of minibatch i."""
        nmb = len(per_learner_args[0])
        self.tables, self.plans = [], []
        for i in range(nmb):
            arr = (PpoArgs * self.G)()
            for g in range(self.G):
                ctypes.memmove(ctypes.byref(arr[g]), ctypes.byref(per_learner_args[g][i]),
                               ctypes.sizeof(PpoArgs))
            t = torch.empty(self._nb, dtype=torch.uint8, device=self.fused[0].flat.device)
            plan = PpoGroupPlan()
            check(self.L.hwy_ppo_group_prepare(arr, self.G, t.data_ptr(), ctypes.byref(plan),
                                               stream_ptr()), "hwy_ppo_group_prepare")
            self.tables.append(t)
            self.plans.append(plan)

    def step(self, i: int) -> None:
        check(self.L.hwy_ppo_group_step(ctypes.byref(self.plans[i]), self.tables[i].data_ptr(),
                                        stream_ptr()), "hwy_ppo_group_step")
