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

from typing import Callable, List, Optional, Sequence

import torch

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
        self._upd = None  # (key, GroupStep, graph)
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

    def _steps(self, tiles) -> None:
        buf, env = self.buf, self.env
        GE = self.G * self.E
        obs_shape = env.obs_buf.shape[1:]
        for t in range(self.T):
            self.act(buf.states[t], (buf.actions[t], buf.pre_tanh[t], buf.log_probs[t],
                                     buf.values[t]), noise=buf.noise[t], tiles=tiles)
            env.step_into(buf.actions[t], buf.states[t + 1].view(GE, *obs_shape), buf.rewards[t],
                          buf.terminated[t], buf.truncated[t], buf.ep_return[t],
                          buf.ep_length[t])
        buf.finish_dones()

    def rollout(self) -> None:
        """T steps of every experiment (LockstepRollout's order: act, then env step, per t);
        captured as one HIP graph once its launch arguments repeat."""
        self._draw_noise()
        tiles = self.act.tiles()  # also syncs acting-only tile images, outside any capture
        if not self.use_graphs:
            self._steps(tiles)
            return
        key = (self.env._handle.value, self.env.launch_version, tuple(tiles))
        if self._roll_graph is not None and key == self._roll_key:
            self.stats["rollout_replay"] += 1
            self._roll_graph.replay()
            return
        if key != self._roll_seen:  # first rollout at these arguments: eager (builds the tables)
            self.stats["rollout_eager"] += 1
            self._roll_seen = key
            self._steps(tiles)
            return
        self.stats["rollout_capture"] += 1
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                self._steps(tiles)
        torch.cuda.current_stream().wait_stream(s)
        self._roll_graph, self._roll_key = g, key
        g.replay()

    # ------------------------------------------------------------------ update
    def bootstrap_values(self) -> torch.Tensor:
        """V(states[T]) of every experiment (PPOAgent.value: the deterministic act launch)."""
        self.act(self.buf.states[self.T], self._boot, noise=None)
        return self._boot[3]

    def update(self, return_metrics: bool = True):
        """PPOAgent.update_rollout for every experiment at once (ppo/agent.py's batched update:
        GAE, per-experiment advantage normalisation and permutation, epochs x minibatches of the
        fused step, metrics)."""
        from hwy import ops
        from hwy.ppo_native import GroupStep

        buf, G, E, T = self.buf, self.G, self.E, self.T
        n, GE = T * E, G * E
        adv, ret = ops.gae(buf.rewards, buf.dones, buf.values, self.bootstrap_values(),
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
        if self._upd is None or self._upd[0] != (tuple(id(F) for F in fused), mb, nmb):
            # static inputs of the captured steps (FusedPPO's _static_bufs): advantages,
            # returns and the mapped permutations are copied in every update
            adv_g = torch.empty(T * GE, device=self.dev)
            ret_g = torch.empty(T * GE, device=self.dev)
            idx = torch.empty(G, n, dtype=torch.int64, device=self.dev)
            self._upd = [(tuple(id(F) for F in fused), mb, nmb), GroupStep(fused), None, adv_g,
                         idx, None, ret_g]
        _, step, graph, adv_grp, idx_all, bound, ret_flat = self._upd
        adv3 = adv_grp.view(T, G, E)
        perms = self._perms if getattr(self, "_perms", None) is not None else \
            torch.empty(G, n, dtype=torch.int64, device=self.dev)
        self._perms = perms
        for g, ag in enumerate(self.agents):
            # the solo update_rollout's order on this experiment's generator and samples
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
        if bound != key:  # the learners' argument structs and the device tables, once per key
            self.stats["update_prepare"] += 1
            args = [[F._args(states, pre, old_lp, adv_grp, ret_flat,
                             idx_all[g].data_ptr() + i * mb * 8) for i in range(nmb)]
                    for g, F in enumerate(fused)]
            step.prepare(args)
            graph = None
            self._upd[2] = None
            self._upd[5] = key
            self._args = args
        args = self._args
        for F, a in zip(fused, args):
            F._last_args, F._last_inputs = a, (states, pre, old_lp, adv_grp, ret_flat, idx_all)
            F.counters[1].zero_()
            F.sync_params(a[0])  # FusedPPO.run's tile-image refresh
        epochs = self.agents[0].epochs
        if not self.use_graphs:
            for _ in range(epochs):
                for i in range(nmb):
                    step.step(i)
        else:
            if graph is None:  # one epoch's minibatch steps as one graph (FusedPPO._capture)
                self.stats["update_capture"] += 1
                graph = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    with torch.cuda.graph(graph, stream=s):
                        for i in range(nmb):
                            step.step(i)
                torch.cuda.current_stream().wait_stream(s)
                self._upd[2] = graph
            for _ in range(epochs):
                graph.replay()
        out = []
        for g, (ag, F) in enumerate(zip(self.agents, fused)):
            F._tiles_version = F._param_versions()
            ag.updates += 1
            if return_metrics:
                vals = buf.values[:, g * E:(g + 1) * E].reshape(n)
                rets = ret[:, g * E:(g + 1) * E].reshape(n)
                out.append(ag._finish_metrics(F.metrics, sizes, vals, rets,
                                              deferred=return_metrics == "deferred"))
        self.iterations += 1
        buf.states[0].copy_(buf.states[T])
        return out if return_metrics else None

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
