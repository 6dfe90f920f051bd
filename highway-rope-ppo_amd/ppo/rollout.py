"""Lockstep rollout of T policy steps over E device envs (the collection half of
training/routine.py:121-160, batched), optionally replayed as one HIP graph.

Per step t: ActorCritic.act on buf.states[t] with the rollout's pre-drawn noise (one hwy_ppo_act
launch writing the action / pre-tanh / log-prob / value rows), then hwy_step writing the next
observation, reward, flags and episode statistics straight into buf's row t (+1).  The 2T
launches have fixed arguments between updates, so from the second rollout on they are captured
once and replayed as a single graph: no host work per step and ~1 us instead of ~6 us between
dependent launches.  The graph is re-captured whenever something it baked in changes: the env
handle or its launch configuration (seed schedule, fused PE table), the acting weights (the
update's tile image or the flat parameters), or the buffers.
"""

from __future__ import annotations

from typing import Optional

import torch

from utils.graphs import capture as graph_capture


class LockstepRollout:
    def __init__(self, agent, env, buf, use_graph: bool = True):
        self.agent = agent
        self.env = env.unwrapped if hasattr(env, "unwrapped") else env
        self.buf = buf
        self.use_graph = bool(use_graph) and self.buf.states.is_cuda
        self._graph: Optional[torch.cuda.CUDAGraph] = None
        self._key = None
        self._seen = None  # key of the last eager run (capture once a key repeats)
        # the env step through a launch-parameter table (hwy_step_group with one handle): the
        # kernel reads the handle's configuration from device memory instead of its kernel
        # arguments, which spares its scalar registers (SGPR spills 114 -> 9) and runs ~4 %
        # faster per step, with the same results (tools/probe_step_group1.py)
        from hwy.vec_env import GroupEnvStep

        self._envstep = GroupEnvStep([self.env]) if hasattr(self.env, "_handle") else None

    def _launch_key(self):
        from hwy.ppo_native import flat_params

        ag, env, buf = self.agent, self.env, self.buf
        flat = flat_params(ag)[0] if ag.backend != "torch" else None
        F = getattr(ag, "_fused", None)
        tiles = F.current_tiles(flat) if (F is not None and flat is not None) else None
        params = tuple(p.data_ptr() for p in ag.actor_critic.parameters())
        return (env._handle.value, getattr(env, "launch_version", 0), tiles, params,
                buf.states.data_ptr(), buf.noise.data_ptr(), buf.T, buf.E)

    def _steps(self) -> None:
        ag, env, buf = self.agent, self.env, self.buf
        E = buf.E
        obs_shape = env.obs_buf.shape[1:]
        for t in range(buf.T):
            ag.select_action(buf.states[t], out=(buf.actions[t], buf.pre_tanh[t],
                                                 buf.log_probs[t], buf.values[t]),
                             noise=buf.noise[t])
            io = (buf.actions[t], buf.states[t + 1].view(E, *obs_shape), buf.rewards[t],
                  buf.terminated[t], buf.truncated[t], buf.ep_return[t], buf.ep_length[t])
            if self._envstep is not None:
                self._envstep.launch([io])
            else:
                env.step_into(*io)
        buf.finish_dones()

    def run(self) -> None:
        """One rollout into buf (rows 0..T-1, states[1..T]); buf.states[0] holds the first obs."""
        self.buf.draw_noise(self.agent.generator)
        if not self.use_graph:
            self._steps()
            return
        key = self._launch_key()
        if self._graph is not None and key == self._key:
            self._graph.replay()
            return
        if key != self._seen:  # first rollout at these arguments: eager (allocations, set-up)
            self._seen = key
            self._steps()
            return
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with graph_capture(g, stream=s):
                self._steps()
        torch.cuda.current_stream().wait_stream(s)
        self._graph, self._key = g, key
        g.replay()
