"""ExperimentRunner (reference experiments/runner.py:19-155) on the MI355X env.

Same launch sequence and status dict: acquire device -> seed -> logger -> make_env ->
``env.to(device)`` when the wrapper has it -> state/action dims -> PPOAgent ->
train_with_experiment_name -> {"status": "COMPLETED"|"FAILED", ...}.  Experiment.extra may carry
``num_envs`` (lockstep envs, > 1 selects the vectorised loop) and ``num_minibatches``.

Launched under torchrun (WORLD_SIZE > 1) one experiment spans the ranks, one GPU each: the
runner joins the process group (RCCL, or ``HWY_DIST_BACKEND``), gives rank r the envs
r*num_envs.. of world*num_envs on the shared seed schedule and hands the group to PPOAgent
(weights broadcast from rank 0, gradients and advantage statistics all-reduced).  Rank 0 logs,
evaluates and writes the artifacts; the other ranks' results carry ``rank``.  The reference
instead runs one single-GPU process per experiment and oversubscribes the GPUs
(SURVEY.md §8(f)).
"""

from __future__ import annotations

import logging
import time
import traceback
from typing import Any, Dict

import numpy as np
import torch

from hwy.gym import spaces
from ppo.agent import PPOAgent
from training.routine import train_with_experiment_name
from utils.logging_utils import setup_experiment_logger
from utils.reproducibility import set_random_seeds

from .config import Experiment
from .wrappers import make_env


class DevicePool:
    """One HIP device per process (torch.distributed rank or LOCAL_RANK), not oversubscribed."""

    def __init__(self, device: Any = None):
        import os

        if device is None and torch.cuda.is_available():
            device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0))
                                  % max(1, torch.cuda.device_count()))
        self.device = torch.device(device) if device is not None else torch.device("cpu")

    def acquire(self):
        import contextlib

        @contextlib.contextmanager
        def _cm():
            yield self.device

        return _cm()


class ExperimentRunner:
    def __init__(self, base_env_config: dict, device_pool=None):
        self.base_config = base_env_config
        self.pool = device_pool or DevicePool()

    @staticmethod
    def _process_group(device):
        """The torchrun world as a process group, or None for a single-process launch."""
        import os

        import torch.distributed as dist

        if int(os.environ.get("WORLD_SIZE", "1")) <= 1 and not dist.is_initialized():
            return None
        if not dist.is_initialized():
            backend = os.environ.get("HWY_DIST_BACKEND") or (
                "nccl" if device.type == "cuda" else "gloo")
            if backend == "nccl":
                torch.cuda.set_device(device)
                dist.init_process_group("nccl", device_id=device)
            else:
                dist.init_process_group(backend)
        return dist.group.WORLD if dist.get_world_size() > 1 else None

    def _create_agent(self, state_dim, action_dim, hp, logger, device, extra=None,
                      process_group=None, seed=None):
        extra = extra or {}
        return PPOAgent(state_dim=state_dim, action_dim=action_dim, lr=hp.lr, gamma=hp.gamma,
                        lam=hp.lam, eps_clip=hp.clip_eps, value_coef=hp.value_coef,
                        entropy_coef=hp.entropy_coef, max_grad_norm=hp.max_grad_norm,
                        epochs=hp.epochs, batch_size=hp.batch_size, hidden_dim=hp.hidden_dim,
                        logger=logger, device=device, process_group=process_group,
                        num_minibatches=extra.get("num_minibatches"), seed=seed)

    def launch(self, exp: Experiment) -> Dict[str, Any]:
        results: Dict[str, Any] = {"experiment_name": exp.name, "status": "FAILED"}
        t0 = time.time()
        logger = None
        try:
            with self.pool.acquire() as device:
                group = self._process_group(device)
                rank, world = ((torch.distributed.get_rank(group),
                                torch.distributed.get_world_size(group))
                               if group is not None else (0, 1))
                set_random_seeds(exp.seed)
                if rank == 0:
                    logger = setup_experiment_logger(exp.name)
                else:
                    results["rank"] = rank
                    logger = logging.getLogger(f"hwy.{exp.name}.rank{rank}")
                    logger.addHandler(logging.NullHandler())
                    logger.propagate = False
                logger.info(f"[{exp.name}] Acquired device: {device} | Seed: {exp.seed}")
                logger.info(f"[{exp.name}] Condition: {exp.condition.name} | HPs: {exp.hp}")
                env = None
                agent = None
                try:
                    overrides = dict(exp.env_config_overrides)
                    if "num_envs" in exp.extra:
                        overrides.setdefault("num_envs", exp.extra["num_envs"])
                    if device.type == "cuda":
                        overrides.setdefault("device", device)
                    if group is not None:
                        e = int(overrides.get("num_envs", 1))
                        if e <= 1:
                            raise ValueError("a multi-rank experiment needs extra['num_envs'] > 1")
                        overrides.update(env_offset=rank * e, global_envs=world * e)
                    env = make_env(exp.condition, self.base_config, d_embed=exp.hp.d_embed,
                                   env_overrides=overrides)
                    if hasattr(env, "to") and callable(env.to):
                        env = env.to(device)
                    if not isinstance(env.observation_space, spaces.Box):
                        raise TypeError(f"Unsupported observation space: {type(env.observation_space)}")
                    state_dim = int(np.prod(env.observation_space.shape))
                    action_dim = env.action_space.shape[0]
                    logger.info(f"[{exp.name}] state_dim={state_dim}, action_dim={action_dim}")
                    # every rank seeds the global RNGs with exp.seed (the RankPE table and the
                    # initial weights must agree), but each rank's sampling generator gets its
                    # own stream, so global env r*E+e does not replay env e's exploration noise
                    agent_seed = None if group is None else exp.seed * 1000003 + rank
                    agent = self._create_agent(state_dim, action_dim, exp.hp, logger, device,
                                               exp.extra, process_group=group, seed=agent_seed)
                    rewards, avg_rewards, metrics = train_with_experiment_name(
                        env=env, agent=agent, max_episodes=exp.max_episodes,
                        target_reward=exp.target_reward,
                        log_interval=exp.extra.get("log_interval", 20),
                        eval_interval=exp.extra.get("eval_interval", 50),
                        steps_per_update=exp.hp.steps_per_update, experiment_name=exp.name,
                        exp_seed=exp.seed, logger=logger)
                    results.update(status="COMPLETED", rewards=rewards, avg_rewards=avg_rewards,
                                   metrics_history=metrics)
                except Exception as e:
                    logger.error(f"[{exp.name}] Experiment execution failed!", exc_info=True)
                    results["error_message"] = str(e)
                    results["error_traceback"] = traceback.format_exc()
                finally:
                    # graphs holding RCCL collectives are freed while the communicator lives
                    if agent is not None and getattr(agent, "_fused", None) is not None:
                        agent._fused.release_graphs()
                    if env is not None:
                        env.close()
        except Exception as e:
            results["error_message"] = str(e)
            results["error_traceback"] = traceback.format_exc()
        results["duration_seconds"] = time.time() - t0
        if logger:
            logger.info(f"[{exp.name}] Run finished. Status: {results['status']}. "
                        f"Duration: {results['duration_seconds']:.2f}s")
        logging.shutdown()
        return results

    def launch_group(self, exps) -> list:
        """launch() for experiments that differ only in their seed (a sweep cell's seeds), run
        as ONE ExperimentGroup on this runner's device (ppo/group.py: the experiments batched into
        the env, acting and minibatch-step launches; each bit-identical to its solo launch()).
        The reference runs such a cell as len(exps) separate processes oversubscribing the GPUs
        (main.py:188-242, utils/device_pool.py:44-72).  Needs the vectorised loop
        (extra["num_envs"] > 1) and the fused HIP learner; returns one status dict per experiment,
        in order."""
        return self.launch_batch([exps])[0]

    def launch_batch(self, cells) -> list:
        """launch_group for several cells at once: each cell (experiments that differ only in
        seed) becomes an ExperimentGroup, and the cells, which must share envs per experiment,
        rollout length and hidden width (e.g. a sweep's four h256 conditions, whose state dims
        differ), are stepped together by one GroupBatch: one acting launch, one env launch and
        one grouped minibatch step for all their learners.  Every experiment stays bit-identical
        to its solo launch().  Returns one list of status dicts per cell."""
        import math

        from ppo.group import GroupBatch, build_group
        from training.routine import train_batch

        cells = [list(c) for c in cells]
        t0 = time.time()
        for exps in cells:
            key = {(e.condition, repr(e.hp), repr(sorted(e.extra.items())),
                    repr(e.env_config_overrides), e.max_episodes, e.target_reward) for e in exps}
            if len(key) != 1:
                raise ValueError("launch_group: the experiments must differ only in seed and name")
            if int(exps[0].extra.get("num_envs", 1)) <= 1:
                raise ValueError("launch_group needs extra['num_envs'] > 1 (the vectorised loop)")
        first = [c[0] for c in cells]
        shared = {(int(e.extra.get("num_envs", 1)), e.hp.steps_per_update, e.hp.hidden_dim,
                   e.max_episodes, e.target_reward, e.extra.get("eval_interval", 50))
                  for e in first}
        if len(shared) != 1:
            raise ValueError("launch_batch: the cells must share num_envs, steps_per_update, "
                             "hidden_dim, max_episodes, target_reward and eval_interval")
        results = [[{"experiment_name": e.name, "status": "FAILED"} for e in exps]
                   for exps in cells]
        loggers = []
        groups = []
        try:
            with self.pool.acquire() as device:
                for exps in cells:
                    e0 = exps[0]
                    E = int(e0.extra.get("num_envs", 1))
                    cell_loggers = []
                    for e in exps:
                        set_random_seeds(e.seed)  # as launch() does before the logger
                        lg = setup_experiment_logger(e.name)
                        lg.info(f"[{e.name}] Acquired device: {device} | Seed: {e.seed} | group "
                                f"of {len(exps)}")
                        cell_loggers.append(lg)
                    loggers += cell_loggers
                    T = max(1, math.ceil(e0.hp.steps_per_update / E))
                    lg_iter = iter(cell_loggers)

                    def make_agent(sd, e0=e0, lg_iter=lg_iter):
                        return self._create_agent(sd, 2, e0.hp, next(lg_iter), device, e0.extra)

                    groups.append(build_group(e0.condition, self.base_config,
                                              [e.seed for e in exps], E, T, device, make_agent,
                                              d_embed=e0.hp.d_embed,
                                              env_overrides=e0.env_config_overrides))
                stepper = groups[0] if len(groups) == 1 else GroupBatch(groups)
                e0 = first[0]
                outs = train_batch(stepper, groups, [e.name for c in cells for e in c],
                                   [e.seed for c in cells for e in c],
                                   max_episodes=e0.max_episodes, target_reward=e0.target_reward,
                                   log_interval=e0.extra.get("log_interval", 20),
                                   eval_interval=e0.extra.get("eval_interval", 50),
                                   loggers=loggers)
                flat = [res for cell in results for res in cell]
                for res, (rewards, avg_rewards, metrics) in zip(flat, outs):
                    res.update(status="COMPLETED", rewards=rewards, avg_rewards=avg_rewards,
                               metrics_history=metrics)
        except Exception as ex:
            for cell in results:
                for res in cell:
                    res["error_message"] = str(ex)
                    res["error_traceback"] = traceback.format_exc()
        finally:
            for g in groups:
                g.close()
        for cell in results:
            for res in cell:
                res["duration_seconds"] = time.time() - t0
        logging.shutdown()
        return results
