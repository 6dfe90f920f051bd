"""ExperimentGroup: G independent PPO experiments of one condition on one GPU, stepped together.

The reference runs a sweep as one process per experiment (experiments/runner.py:46-155 under
main.py:188-242's joblib / SLURM fan-out, utils/device_pool.py:44-72 oversubscribing each GPU
16x).  At the reference's own update statistics (E = 16 envs x T = 128 steps = 2,048 samples,
minibatches of 64) one experiment is far too small to fill an MI355X: every launch of its rollout
and update runs a handful of workgroups.  A group batches G such experiments -- a condition's
seeds -- into the launches themselves:

  * one env handle of G*E envs, experiment g owning envs [g*E, (g+1)*E) with its own episode
    seed schedule (hwy_set_seed_groups) and, for RankPE, its own rank table;
  * one acting launch per rollout step for all G policies (hwy_ppo_group_act);
  * one GAE launch over the [T, G*E] rollout;
  * per minibatch step four launches for all G learners (hwy_ppo_group_step), each learner
    reading its own minibatch through its own permutation mapped into the grouped rollout.

Every experiment keeps its own weights, Adam state, torch generator (sampling noise and the
minibatch permutation) and advantage normalisation, drawn in its solo run's order, and the
kernels run the solo calls' bodies per learner, so each experiment is bit for bit its solo run
(training/routine.py's _train_vector with the same seed): tests/test_group_gpu.py.
"""

from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch

from utils.graphs import capture as graph_capture

from .agent import RolloutBuffer


class ExperimentGroup:
    def __init__(self, agents: Sequence, env, seeds: Sequence[int], envs_per_experiment: int,
                 rollout_len: int, use_graphs: bool = True, rank_tables=None):
        from hwy.ppo_native import GroupAct

        self.agents = list(agents)
        self.G, self.E, self.T = len(self.agents), int(envs_per_experiment), int(rollout_len)
        self.env = env.unwrapped if hasattr(env, "unwrapped") else env
        if self.env.num_envs != self.G * self.E:
            raise ValueError(f"the group env needs {self.G} x {self.E} envs, has {self.env.num_envs}")
        if len(seeds) != self.G:
            raise ValueError("one seed per experiment")
        a0 = self.agents[0]
        dims = {(ag.actor_critic.shared[0].weight.shape, ag.epochs, ag.batch_size,
                 ag.num_minibatches) for ag in self.agents}
        if len(dims) != 1 or any(ag.device != a0.device for ag in self.agents):
            raise ValueError("a group's experiments share learner dims, epochs, batch size, device")
        self.dev = a0.device
        self.seeds = [int(s) for s in seeds]
        # per-experiment episode seed schedules: group g as a solo handle of E envs seeded with
        # set_seed_schedule(seeds[g]) (training/routine.py:_train_vector)
        self.env.set_seed_groups(self.seeds, self.E)
        if rank_tables is not None:
            import numpy as np

            self.env.set_pe_table(np.concatenate([np.asarray(t, np.float32).reshape(-1)
                                                  for t in rank_tables]))
        N, Fo = self.env.obs_rows, self.env.obs_features
        self.sd = N * Fo
        self.buf = RolloutBuffer(self.T, self.G * self.E, self.sd, 2, self.dev)
        self.use_graphs = bool(use_graphs)
        self.act = GroupAct(self.agents, self.E)
        GE = self.G * self.E
        # the bootstrap value row's outputs (deterministic act on states[T]); fixed buffers, so
        # their argument tables are prepared once
        self._boot = tuple(torch.empty(*s, device=self.dev) for s in ((GE, 2), (GE, 2), (GE,), (GE,)))
        self._noise_tmp = torch.empty(self.T, self.E, 2, device=self.dev)
        self._roll_graph = None
        self._roll_key = None
        self._roll_seen = None
        self._upd = None  # the update's static inputs and argument structs (pre_update)
        self.iterations = 0
        # how the rollouts / updates were issued (graph replays vs eager runs vs captures, and
        # argument-table preparations): a sweep that keeps re-preparing shows here
        self.stats = {"rollout_replay": 0, "rollout_eager": 0, "rollout_capture": 0,
                      "update_prepare": 0, "update_capture": 0}
        obs, _ = self.env.reset()
        self.buf.states[0].copy_(obs.reshape(GE, self.sd))

    # ------------------------------------------------------------------ rollout
    def _draw_noise(self) -> None:
        """Each experiment's T x E x 2 sampling noise from its own generator, exactly as its
        solo RolloutBuffer.draw_noise draws it."""
        buf, E = self.buf, self.E
        for g, ag in enumerate(self.agents):
            torch.randn(self._noise_tmp.shape, generator=ag.generator, device=self.dev,
                        out=self._noise_tmp)
            buf.noise[:, g * E:(g + 1) * E].copy_(self._noise_tmp)

    def act_rows(self, t: int, deterministic: bool = False):
        """This group's acting rows at rollout step t (GroupAct.rows_of), or, deterministic, the
        bootstrap row states[T] into the fixed bootstrap outputs."""
        buf = self.buf
        if deterministic:
            return self.act.rows_of(buf.states[self.T], self._boot, None)
        return self.act.rows_of(buf.states[t], (buf.actions[t], buf.pre_tanh[t], buf.log_probs[t],
                                                buf.values[t]), buf.noise[t])

    def env_io(self, t: int):
        """step_into's buffers for rollout step t (hwy_step's arguments)."""
        buf, env = self.buf, self.env
        obs_shape = env.obs_buf.shape[1:]
        return (buf.actions[t], buf.states[t + 1].view(self.G * self.E, *obs_shape),
                buf.rewards[t], buf.terminated[t], buf.truncated[t], buf.ep_return[t],
                buf.ep_length[t])

    def env_step(self, t: int) -> None:
        self.env.step_into(*self.env_io(t))

    def _steps(self, tiles) -> None:
        for t in range(self.T):
            self.act.launch(self.act_rows(t), tiles)
            self.env_step(t)
        self.buf.finish_dones()

    def rollout(self) -> None:
        """T steps of every experiment (LockstepRollout's order: act, then env step, per t);
        captured as one HIP graph once its launch arguments repeat."""
        self._draw_noise()
        tiles = self.act.tiles()  # also syncs acting-only tile images, outside any capture
        key = (self.env._handle.value, self.env.launch_version, tuple(tiles))
        self._roll_graph, self._roll_key, self._roll_seen = _graph_run(
            self, self.use_graphs, key, lambda: self._steps(tiles), self._roll_graph,
            self._roll_key, self._roll_seen, "rollout")

    # ------------------------------------------------------------------ update
    def bootstrap_values(self) -> torch.Tensor:
        """V(states[T]) of every experiment (PPOAgent.value: the deterministic act launch)."""
        self.act.launch(self.act_rows(0, deterministic=True))
        return self._boot[3]

    def pre_update(self, last_values: torch.Tensor) -> dict:
        """The update's inputs for every experiment, in its solo update_rollout's order on its
        generator and samples (ppo/agent.py's batched update): GAE over the [T, G*E] rollout,
        each experiment's advantage normalisation and permutation mapped into the grouped
        rollout, the learners' FusedPPO (its Adam state handed over) with its per-update
        refresh (counters, tile image).  Returns the context post_update and the step runner
        use; ctx["args"][g][i] is learner g's PpoArgs of minibatch i, rebuilt only when the
        buffers or hyper-parameters change (ctx["key"])."""
        from hwy import ops

        buf, G, E, T = self.buf, self.G, self.E, self.T
        n, GE = T * E, G * E
        adv, ret = ops.gae(buf.rewards, buf.dones, buf.values, last_values,
                           self.agents[0].gamma, self.agents[0].lam)
        sizes = self.agents[0].minibatch_sizes(n)
        mb, nmb = sizes[0], len(sizes)
        if len(set(sizes)) != 1:
            raise ValueError(f"grouped update needs equal minibatches, got {sorted(set(sizes))}")
        fused = []
        for ag in self.agents:
            if not ag._fused_ok(mb):
                raise ValueError("grouped update needs the fused HIP learner (backend hip/auto)")
            F = ag._fused_for(mb, nmb, n)
            ag._adam_to("fused")
            fused.append(F)
        fkey = (tuple(id(F) for F in fused), mb, nmb)
        if self._upd is None or self._upd[0] != fkey:
            # static inputs of the captured steps (FusedPPO's _static_bufs): advantages,
            # returns and the mapped permutations are copied in every update
            self._upd = [fkey, torch.empty(T * GE, device=self.dev),
                         torch.empty(T * GE, device=self.dev),
                         torch.empty(G, n, dtype=torch.int64, device=self.dev),
                         torch.empty(G, n, dtype=torch.int64, device=self.dev), None, None]
        _, adv_grp, ret_flat, idx_all, perms, bound, args = self._upd
        adv3 = adv_grp.view(T, G, E)
        for g, ag in enumerate(self.agents):
            a = ag.normalize_advantages(adv[:, g * E:(g + 1) * E].reshape(n))
            adv3[:, g].copy_(a.view(T, E))
            torch.randperm(n, device=self.dev, generator=ag.generator, out=perms[g])
        # sample (t, l) of experiment g sits at t*G*E + g*E + l of the grouped rollout
        offs = torch.arange(G, device=self.dev, dtype=torch.int64).mul_(E).view(G, 1)
        torch.add(torch.div(perms, E, rounding_mode="floor") * GE + offs, perms % E, out=idx_all)
        states = buf.states[:T].reshape(T * GE, -1)
        pre = buf.pre_tanh.reshape(T * GE, -1)
        old_lp = buf.log_probs.reshape(T * GE)
        ret_flat.copy_(ret.reshape(T * GE))
        key = (states.data_ptr(), pre.data_ptr(), old_lp.data_ptr(), adv_grp.data_ptr(),
               ret_flat.data_ptr(), idx_all.data_ptr()) + tuple(F._scalar_key() for F in fused)
        if bound != key:
            args = [[F._args(states, pre, old_lp, adv_grp, ret_flat,
                             idx_all[g].data_ptr() + i * mb * 8) for i in range(nmb)]
                    for g, F in enumerate(fused)]
            self._upd[5], self._upd[6] = key, args
        for F, a in zip(fused, args):
            F._last_args, F._last_inputs = a, (states, pre, old_lp, adv_grp, ret_flat, idx_all)
            F.counters[1].zero_()
            F.sync_params(a[0])  # FusedPPO.run's tile-image refresh
        return {"fused": fused, "args": args, "key": key, "sizes": sizes, "nmb": nmb, "ret": ret}

    def post_update(self, ctx: dict, return_metrics=True):
        buf, E, T = self.buf, self.E, self.T
        n = T * E
        out = []
        for g, (ag, F) in enumerate(zip(self.agents, ctx["fused"])):
            F._tiles_version = F._param_versions()
            ag.updates += 1
            if return_metrics:
                vals = buf.values[:, g * E:(g + 1) * E].reshape(n)
                rets = ctx["ret"][:, g * E:(g + 1) * E].reshape(n)
                out.append(ag._finish_metrics(F.metrics, ctx["sizes"], vals, rets,
                                              deferred=return_metrics == "deferred"))
        self.iterations += 1
        buf.states[0].copy_(buf.states[T])
        return out if return_metrics else None

    def update(self, return_metrics: bool = True):
        """PPOAgent.update_rollout for every experiment at once: pre_update, epochs x
        minibatches of the grouped fused step (one graph per epoch), post_update."""
        ctx = self.pre_update(self.bootstrap_values())
        self._steps_runner = _run_group_steps(self, [ctx], getattr(self, "_steps_runner", None))
        return self.post_update(ctx, return_metrics)

    def iteration(self, return_metrics=True):
        """One PPO iteration of every experiment: rollout, then update."""
        self.rollout()
        return self.update(return_metrics)

    def close(self) -> None:
        """Release the grouped env handle and the experiments' own (evaluation template) envs."""
        for e in getattr(self, "solo_envs", []) + [getattr(self, "group_env", self.env)]:
            try:
                e.close()
            except Exception:
                pass

    def episode_returns(self, g: int) -> torch.Tensor:
        """Returns of experiment g's episodes that ended in the last rollout, in (step, env)
        order (training/routine.py:_episode_ends on its [T, E] slice)."""
        E = self.E
        d = self.buf.dones[:, g * E:(g + 1) * E]
        r = self.buf.ep_return[:, g * E:(g + 1) * E]
        return r[d != 0]


def _graph_run(owner, use_graphs, key, steps, graph, gkey, seen, what):
    """LockstepRollout's issue policy for a launch sequence `steps`: replay the captured graph
    when its key repeats, run eagerly the first time a key is seen (allocations, argument
    tables), capture it the second time.  Returns the new (graph, graph key, seen key)."""
    if not use_graphs:
        steps()
        return graph, gkey, seen
    if graph is not None and key == gkey:
        owner.stats[f"{what}_replay"] += 1
        graph.replay()
        return graph, gkey, seen
    if key != seen:
        owner.stats[f"{what}_eager"] += 1
        steps()
        return graph, gkey, key
    owner.stats[f"{what}_capture"] += 1
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with graph_capture(g, stream=s):
            steps()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    return g, key, seen


def _run_group_steps(owner, ctxs, runner):
    """Every epoch's minibatch steps of the learners of `ctxs` (pre_update contexts) as grouped
    launches: one GroupStep over all of them, its tables prepared when any member's arguments
    changed, one epoch captured as a graph and replayed `epochs` times (FusedPPO.run's
    schedule).  runner = (key, GroupStep, graph) kept by the owner between updates."""
    from hwy.ppo_native import GroupStep

    fused = [F for c in ctxs for F in c["fused"]]
    args = [a for c in ctxs for a in c["args"]]
    key = (tuple(id(F) for F in fused),) + tuple(c["key"] for c in ctxs)
    nmb = ctxs[0]["nmb"]
    if any(c["nmb"] != nmb for c in ctxs):
        raise ValueError("grouped learners need the same minibatch count")
    if runner is None or runner[0] != key:
        owner.stats["update_prepare"] += 1
        step = GroupStep(fused)
        step.prepare(args)
        runner = (key, step, None)
    _, step, graph = runner
    epochs = fused[0].agent.epochs
    if not owner.use_graphs:
        for _ in range(epochs):
            for i in range(nmb):
                step.step(i)
        return runner
    if graph is None:  # one epoch's minibatch steps as one graph (FusedPPO._capture)
        owner.stats["update_capture"] += 1
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with graph_capture(graph, stream=s):
                for i in range(nmb):
                    step.step(i)
        torch.cuda.current_stream().wait_stream(s)
        runner = (key, step, graph)
    for _ in range(epochs):
        graph.replay()
    return runner


class GroupBatch:
    """Several ExperimentGroups of one hidden width and the same rows per learner (a sweep's
    cells that differ only in observation layout, e.g. the four h256 cells: no PE, RoPE, DistPE,
    RankPE, whose state dims are 60 or 120) stepped as ONE set of launches: per rollout step one
    acting launch for every learner of every group and one env launch for every group's handle
    (hwy_step_group); per minibatch step one grouped fused step over all their learners (hwy_ppo_group_step takes learners of
    different state dims).  Each experiment stays bit-identical to its solo run: the same
    kernel bodies per learner, each group's own generator order, GAE and normalisation."""

    def __init__(self, groups, use_graphs: bool = True):
        from hwy.ppo_native import GroupAct

        self.groups = list(groups)
        g0 = self.groups[0]
        if any(g.E != g0.E or g.T != g0.T for g in self.groups):
            raise ValueError("a batch's groups share envs per experiment and rollout length")
        self.agents = [a for g in self.groups for a in g.agents]
        self.act = GroupAct(self.agents, g0.E)
        # the groups' env steps as one launch (hwy_step_group): each group's handle alone holds
        # G x E envs -- one wave each, a small part of the GPU -- so n launches in a row would
        # leave most of it idle
        from hwy.vec_env import GroupEnvStep

        self.envstep = GroupEnvStep([g.env for g in self.groups]) if len(self.groups) > 1 else None
        self.use_graphs = bool(use_graphs)
        self.T = g0.T
        self._roll = (None, None, None)
        self._runner = None
        self.stats = {"rollout_replay": 0, "rollout_eager": 0, "rollout_capture": 0,
                      "update_prepare": 0, "update_capture": 0}

    def _rows(self, t, deterministic=False):
        return [r for g in self.groups for r in g.act_rows(t, deterministic)]

    def _steps(self, tiles):
        for t in range(self.T):
            self.act.launch(self._rows(t), tiles)
            if self.envstep is not None:
                self.envstep.launch([g.env_io(t) for g in self.groups])
            else:
                self.groups[0].env_step(t)
        for g in self.groups:
            g.buf.finish_dones()

    def rollout(self) -> None:
        for g in self.groups:
            g._draw_noise()
        tiles = self.act.tiles()
        key = (tuple((g.env._handle.value, g.env.launch_version) for g in self.groups),
               tuple(tiles))
        self._roll = _graph_run(self, self.use_graphs, key, lambda: self._steps(tiles), *self._roll,
                                "rollout")

    def update(self, return_metrics=True):
        self.act.launch(self._rows(0, deterministic=True))  # every group's bootstrap values
        ctxs = [g.pre_update(g._boot[3]) for g in self.groups]
        self._runner = _run_group_steps(self, ctxs, self._runner)
        return [g.post_update(c, return_metrics) for g, c in zip(self.groups, ctxs)]

    def iteration(self, return_metrics=True):
        """One PPO iteration of every experiment of every group: a list per group."""
        self.rollout()
        return self.update(return_metrics)


def build_group(condition, base_config, seeds: Sequence[int], envs_per_experiment: int,
                rollout_len: int, device: torch.device, make_agent: Callable, d_embed=None,
                env_overrides: Optional[dict] = None, use_graphs: bool = True):
    """A group of len(seeds) experiments of one condition, each constructed as
    experiments/runner.py constructs its solo run: set_random_seeds(seed), make_env (whose RankPE
    table draws from the global torch RNG), env.to(device), then ``make_agent(state_dim)`` (the
    PPOAgent, its weights drawn from the global RNG, its generator seeded from it), so every
    experiment's weights, rank table and generator are its solo run's.  The experiments' own
    E-env handles are kept as ``group.solo_envs`` (templates of their evaluation envs)."""
    import copy

    from experiments.wrappers import make_env
    from hwy.ops import PE_RANK
    from utils.reproducibility import set_random_seeds

    E = int(envs_per_experiment)
    ov = copy.deepcopy(env_overrides or {})
    agents, tables, solos = [], [], []
    for s in seeds:
        set_random_seeds(int(s))
        solo = make_env(condition, base_config, d_embed=d_embed,
                        env_overrides=dict(copy.deepcopy(ov), num_envs=E, device=device,
                                           autoreset=True))
        if hasattr(solo, "to") and callable(solo.to):
            solo = solo.to(device)
        base = solo.unwrapped
        t = getattr(base, "_pe_table", None)
        tables.append(None if t is None else t.copy())
        agents.append(make_agent(base.obs_rows * base.obs_features))
        solos.append(solo)
    env = make_env(condition, base_config, d_embed=d_embed,
                   env_overrides=dict(copy.deepcopy(ov), num_envs=len(seeds) * E, device=device,
                                      autoreset=True))
    if hasattr(env, "to") and callable(env.to):
        env = env.to(device)
    rank = env.unwrapped.hwy_config.pe_kind == PE_RANK and tables[0] is not None
    grp = ExperimentGroup(agents, env, seeds, E, rollout_len, use_graphs=use_graphs,
                          rank_tables=tables if rank else None)
    grp.solo_envs = solos
    grp.group_env = env
    return grp
