"""Training entry point (reference training/routine.py:14-297), on the MI355X env.

``train_with_experiment_name`` keeps the reference's signature, return value
``(rewards, avg_rewards, metrics_history)``, artifact names and schemas:
  * artifacts/highway-ppo/checkpoints/ppo_highway_{best,solved}_<exp>.pth  (:104-107, :208-222)
  * artifacts/highway-ppo/training_metrics_<exp>.json with the same keys  (:88-97, :246-251)
  * artifacts/highway-ppo/summary_<exp>.csv, header
    ``experiment,final_reward,max_reward,steps,best_model,plot``          (:282-295)
  * artifacts/highway-ppo/ppo_highway_rewards_<exp>.png                    (:254-279)

Two loops behind it:
  * a one-env facade env (make_env default) runs the reference's loop as written: per-episode
    ``env.reset(seed=exp_seed + episode_num)`` (:127), batch-1 select_action, list memory,
    ``agent.update(last_value)`` every ``steps_per_update`` steps;
  * a HighwayVecEnv (``num_envs`` > 1) runs E lockstep envs with in-kernel autoreset on the
    same seed schedule (env e's k-th episode gets exp_seed + 1 + e + E*k, = exp_seed +
    episode_num for E = 1), a device RolloutBuffer of T = ceil(steps_per_update / E) steps, and
    ``agent.update_rollout``.  Episode bookkeeping (logging / eval every ``eval_interval``
    completed episodes, best / solved checkpoints, moving average over the last 10 evals) follows
    the reference, with completed episodes counted in env order within each step.
``evaluate`` runs ``num_episodes`` deterministic episodes seeded exp_seed + 1000 + k (:14-29),
as one batched env for the vectorised path.
"""

from __future__ import annotations

import json
import logging
import math
import os
import time

import numpy as np
import torch

from utils.logging_utils import ensure_artifacts_dir, setup_experiment_logger


def _is_vector(env) -> bool:
    return bool(getattr(env.unwrapped, "is_vector_env", False))


def _flat_dim(env) -> int:
    return int(np.prod(env.observation_space.shape))


# ---------------------------------------------------------------------------------- evaluation
def evaluate(env, agent, num_episodes=10, render=False, exp_seed: int = 0):
    """Mean return of deterministic episodes seeded exp_seed + 1000 + k."""
    if _is_vector(env):
        return _evaluate_vector(env, agent, num_episodes, exp_seed)
    totals = []
    for ep in range(num_episodes):
        state, _ = env.reset(seed=exp_seed + 1000 + ep)
        flat = state.reshape(-1)
        done, ep_reward = False, 0.0
        while not done:
            action, _, _, _ = agent.select_action(flat, deterministic=True)
            nxt, reward, terminated, truncated, _ = env.step(action)
            done = terminated or truncated
            flat = nxt.reshape(-1)
            ep_reward += reward
        totals.append(ep_reward)
    return float(np.mean(totals))


def _eval_env_like(env, num_episodes: int):
    """A num_episodes-wide copy of env (same config and fused wrapper), no autoreset."""
    from hwy.vec_env import HighwayVecEnv

    base = env.unwrapped
    cfg = base.hwy_config
    ev = HighwayVecEnv(base.config, num_envs=num_episodes, device=base.device, autoreset=False,
                       pe_kind=cfg.pe_kind, d_embed=cfg.d_embed, ego_idx=cfg.ego_idx,
                       pe_max_dist=cfg.pe_max_dist, pe_table=base._pe_table)
    return ev


def _eval_key(agent, num_episodes, exp_seed):
    """Identity of a deterministic evaluation: the same weights (no update since, no torch-side
    parameter write) on the same seeds give the same return, bit for bit."""
    params = tuple((p.data_ptr(), p._version) for p in agent.actor_critic.parameters())
    # on the fused path every p.data is a view of one flat buffer: writes through that buffer
    # (the fused optimizer, a copy into it) bump only the buffer's counter
    flat = getattr(agent, "_flat", None)
    flat_v = (flat[0].data_ptr(), flat[0]._version) if flat is not None else None
    return (getattr(agent, "updates", None), params, flat_v, num_episodes, exp_seed)


def _evaluate_vector(env, agent, num_episodes, exp_seed):
    # With thousands of lockstep envs many eval points (every eval_interval completed episodes)
    # fall between two updates; the evaluation is deterministic, so a repeat at unchanged
    # weights reuses the last result instead of re-running the episodes.
    key = _eval_key(agent, num_episodes, exp_seed)
    memo = getattr(env.unwrapped, "_eval_memo", None)
    if memo is not None and memo[0] == key and key[0] is not None:
        return memo[1]
    r = _run_eval_vector(env, agent, num_episodes, exp_seed)
    env.unwrapped._eval_memo = (key, r)
    return r


def _run_eval_vector(env, agent, num_episodes, exp_seed):
    cache = getattr(env.unwrapped, "_eval_envs", None)
    if cache is None:
        cache = {}
        env.unwrapped._eval_envs = cache
    ev = cache.get(num_episodes)
    if ev is None:
        ev = cache[num_episodes] = _eval_env_like(env, num_episodes)
    dev = ev.device
    seeds = torch.arange(num_episodes, device=dev, dtype=torch.int64) + (exp_seed + 1000)
    obs, _ = ev.reset(seeds=seeds)
    alive = torch.ones(num_episodes, dtype=torch.bool, device=dev)
    total = torch.zeros(num_episodes, dtype=torch.float64, device=dev)
    for k in range(ev.max_episode_steps + 1):
        a, _, _, _ = agent.select_action(obs.reshape(num_episodes, -1), deterministic=True)
        obs, r, te, tr, _ = ev.step(a.contiguous())
        total += torch.where(alive, r.double(), torch.zeros_like(total))
        alive &= ~(te.bool() | tr.bool())
        # the host learns "all done" every 8 steps (one sync instead of eight): the steps after
        # every episode ended add nothing to total (alive is all False), so the result is the same
        if k % 8 == 7 and not bool(alive.any()):
            break
    return float(total.mean().item())


def evaluate_many(items, num_episodes=5):
    """evaluate(env, agent, num_episodes, exp_seed) for every (env, agent, exp_seed) of `items`,
    each result exactly what evaluate returns for it alone: the evaluations that are not memoised
    run together, one grouped acting launch (hwy_ppo_group_act) and one grouped env launch
    (hwy_step_group) per step over all their evaluation envs, the same kernels and the same
    per-episode float64 sums as the solo loop.  Falls back to one evaluate per item where the
    items cannot share launches (torch acting, mixed hidden widths, single items)."""
    out = [None] * len(items)
    todo = []
    for i, (env, agent, seed) in enumerate(items):
        key = _eval_key(agent, num_episodes, seed)
        memo = getattr(env.unwrapped, "_eval_memo", None)
        if memo is not None and memo[0] == key and key[0] is not None:
            out[i] = memo[1]
        else:
            todo.append(i)
    groups = {}
    for i in todo:
        env, agent, _ = items[i]
        ok = (_is_vector(env) and getattr(agent, "backend", "torch") != "torch"
              and agent.device.type == "cuda")
        H = agent.actor_critic.shared[0].weight.shape[0] if ok else None
        groups.setdefault(H, []).append(i)
    for H, idx in groups.items():
        if H is None or len(idx) < 2:
            for i in idx:
                out[i] = evaluate(items[i][0], items[i][1], num_episodes=num_episodes,
                                  exp_seed=items[i][2])
            continue
        res = _run_eval_group([items[i] for i in idx], num_episodes)
        for i, r in zip(idx, res):
            env, agent, seed = items[i]
            env.unwrapped._eval_memo = (_eval_key(agent, num_episodes, seed), r)
            out[i] = r
    return out


def _run_eval_group(items, num_episodes):
    """_run_eval_vector for several experiments in lockstep (evaluate_many)."""
    from hwy.ppo_native import GroupAct
    from hwy.vec_env import GroupEnvStep

    evs, rows = [], []
    n, k = num_episodes, len(items)
    agents = [a for _, a, _ in items]
    for env, agent, seed in items:
        cache = getattr(env.unwrapped, "_eval_envs", None)
        if cache is None:
            cache = {}
            env.unwrapped._eval_envs = cache
        ev = cache.get(n)
        if ev is None:
            ev = cache[n] = _eval_env_like(env, n)
        evs.append(ev)
    dev = evs[0].device
    act = GroupAct(agents, n)
    tiles = act.tiles()
    if any((t is None) != (tiles[0] is None) for t in tiles):  # one acting kernel per launch
        return [_run_eval_vector(env, agent, n, seed) for env, agent, seed in items]
    rew = torch.empty(k * n, device=dev)
    te = torch.empty(k * n, dtype=torch.uint8, device=dev)
    tr = torch.empty(k * n, dtype=torch.uint8, device=dev)
    ios, keep = [], []  # keep: the act outputs the kernels write through raw addresses
    for j, ((env, agent, seed), ev) in enumerate(zip(items, evs)):
        seeds = torch.arange(n, device=dev, dtype=torch.int64) + (seed + 1000)
        obs, _ = ev.reset(seeds=seeds)  # the eval handle's obs_buf, read and rewritten in place
        a = torch.empty(n, 2, device=dev)
        pre = torch.empty(n, 2, device=dev)
        lp = torch.empty(n, device=dev)
        val = torch.empty(n, device=dev)
        sl = slice(j * n, (j + 1) * n)
        keep.append((a, pre, lp, val))
        rows.append((obs.data_ptr(), None, a.data_ptr(), pre.data_ptr(), lp.data_ptr(),
                     val.data_ptr()))
        ios.append((a, obs, rew[sl], te[sl], tr[sl], None, None))
    step = GroupEnvStep(evs)
    alive = torch.ones(k * n, dtype=torch.bool, device=dev)
    total = torch.zeros(k * n, dtype=torch.float64, device=dev)
    for s_ in range(max(ev.max_episode_steps for ev in evs) + 1):
        act.launch(rows, tiles)
        step.launch(ios)
        total += torch.where(alive, rew.double(), torch.zeros_like(total))
        alive &= ~(te.bool() | tr.bool())
        if s_ % 8 == 7 and not bool(alive.any()):
            break
    res = [float(total[j * n:(j + 1) * n].mean().item()) for j in range(k)]
    del keep
    return res


# ---------------------------------------------------------------------------------- artifacts
def _save_artifacts(artifacts_dir, checkpoint_dir, experiment_name, metrics_history,
                    training_episodes, episode_rewards, eval_episodes, rewards, avg_rewards,
                    target_reward, total_steps, logger, exp_prefix):
    metrics_path = os.path.join(artifacts_dir, f"training_metrics_{experiment_name}.json")
    with open(metrics_path, "w") as f:
        json.dump(metrics_history, f, indent=2)
    logger.info(f"{exp_prefix} Metrics saved to {metrics_path}")
    plot_path = os.path.join(artifacts_dir, f"ppo_highway_rewards_{experiment_name}.png")
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        plt.figure(figsize=(12, 8))
        plt.plot(training_episodes, episode_rewards, alpha=0.3, label="Training Reward", color="gray")
        if len(episode_rewards) > 20:
            sm = np.convolve(episode_rewards, np.ones(20) / 20, mode="valid")
            plt.plot(training_episodes[19:], sm, label="Training (Moving Avg)")
        plt.plot(eval_episodes, rewards, "ro-", label="Eval Reward")
        plt.plot(eval_episodes, avg_rewards, "go-", label="Eval Moving Avg")
        plt.axhline(y=target_reward, color="r", linestyle="--", label="Target Reward")
        plt.xlabel("Episode")
        plt.ylabel("Reward")
        plt.title(f"Training Progress ({experiment_name})")
        plt.legend()
        plt.grid(alpha=0.3)
        plt.savefig(plot_path, bbox_inches="tight")
        plt.close()
        logger.info(f"{exp_prefix} Training plot saved to {plot_path}")
    except Exception as e:  # plotting is cosmetic
        logger.warning(f"{exp_prefix} plot failed: {e}")
    csv_path = os.path.join(artifacts_dir, f"summary_{experiment_name}.csv")
    best_model_path = os.path.join(checkpoint_dir, f"ppo_highway_best_{experiment_name}.pth")
    with open(csv_path, "w") as f:
        f.write("experiment,final_reward,max_reward,steps,best_model,plot\n")
        f.write(f"{experiment_name},{avg_rewards[-1]:.4f},{max(avg_rewards):.4f},{total_steps},"
                f"{best_model_path},{os.path.basename(plot_path)}\n")
    logger.info(f"{exp_prefix} Summary CSV saved to {csv_path}")


class _EvalTracker:
    """Eval / moving-average / checkpoint bookkeeping of routine.py:172-222."""

    def __init__(self, env, agent, exp_seed, target_reward, checkpoint_dir, experiment_name,
                 metrics_history, logger, exp_prefix, start_time):
        self.env, self.agent, self.exp_seed = env, agent, exp_seed
        self.target_reward = target_reward
        self.checkpoint_dir, self.name = checkpoint_dir, experiment_name
        self.mh, self.logger, self.prefix, self.t0 = metrics_history, logger, exp_prefix, start_time
        self.rewards, self.avg_rewards, self.eval_episodes = [], [], [0]
        self.best = -float("inf")
        self.solved = False

    def initial(self, r=None):
        if r is None:
            r = evaluate(self.env, self.agent, num_episodes=5, exp_seed=self.exp_seed)
        self.rewards.append(r)
        self.avg_rewards.append(r)
        self.mh["eval_rewards"].append(r)
        self.mh["avg_eval_rewards"].append(r)
        self.mh["eval_episode_numbers"].append(0)
        self.mh["timestamps"].append(0)
        self.logger.info(f"{self.prefix} initial_eval reward={r:.2f}")

    def on_episode(self, episode_num, r=None):
        """r: the evaluation's result when the caller ran it (evaluate_many), else evaluated here."""
        self.logger.info(f"{self.prefix} Evaluating at episode {episode_num}...")
        if r is None:
            r = evaluate(self.env, self.agent, num_episodes=5, exp_seed=self.exp_seed)
        self.rewards.append(r)
        self.eval_episodes.append(episode_num)
        elapsed = time.time() - self.t0
        avg = float(np.mean(self.rewards[-10:])) if len(self.rewards) >= 10 else float(np.mean(self.rewards))
        self.avg_rewards.append(avg)
        self.mh["eval_rewards"].append(r)
        self.mh["avg_eval_rewards"].append(avg)
        self.mh["eval_episode_numbers"].append(episode_num)
        self.mh["timestamps"].append(elapsed)
        self.logger.info("%s eval episode=%d reward=%.2f avg_reward=%.2f time=%.2fs", self.prefix,
                         episode_num, r, avg, elapsed)
        if avg >= self.target_reward and not self.solved and len(self.rewards) >= 10:
            self.logger.info(f"{self.prefix} Environment solved in {episode_num} episodes! avg reward={avg:.2f}")
            self.agent.save(os.path.join(self.checkpoint_dir, f"ppo_highway_solved_{self.name}.pth"))
            self.solved = True
        if avg > self.best:
            self.best = avg
            self.agent.save(os.path.join(self.checkpoint_dir, f"ppo_highway_best_{self.name}.pth"))
            self.logger.info(f"{self.prefix} New best model saved, avg reward={self.best:.2f}")


# ---------------------------------------------------------------------------------- training
def train_with_experiment_name(env, agent, max_episodes=500, target_reward=0.0, log_interval=20,
                               eval_interval=50, steps_per_update=2048, experiment_name="",
                               exp_seed: int = 0, logger=None):
    if logger is None:
        logger = setup_experiment_logger(experiment_name)
    exp_prefix = f"[{experiment_name}]" if experiment_name else ""
    logger.info(f"{exp_prefix} Starting training for experiment: {experiment_name}")
    metrics_history = {
        "experiment_name": experiment_name,
        "episode_rewards": [],
        "eval_rewards": [],
        "avg_eval_rewards": [],
        "policy_updates": [],
        "episode_numbers": [],
        "eval_episode_numbers": [],
        "timestamps": [],
    }
    start_time = time.time()
    artifacts_dir = ensure_artifacts_dir()
    checkpoint_dir = os.path.join(artifacts_dir, "checkpoints")
    os.makedirs(checkpoint_dir, exist_ok=True)
    tracker = _EvalTracker(env, agent, exp_seed, target_reward, checkpoint_dir, experiment_name,
                           metrics_history, logger, exp_prefix, start_time)
    rank, _ = _rank_world(getattr(agent, "_dist", None))
    if rank == 0:
        logger.info(f"{exp_prefix} Performing initial evaluation...")
        tracker.initial()
    if not _is_vector(env) and getattr(agent, "_dist", None) is not None:
        raise ValueError("a process group needs the vectorised env (num_envs > 1)")
    loop = _train_vector if _is_vector(env) else _train_single
    episode_rewards, training_episodes, total_steps = loop(
        env, agent, max_episodes, log_interval, eval_interval, steps_per_update, exp_seed, logger,
        exp_prefix, metrics_history, tracker, start_time)
    if rank != 0:
        return tracker.rewards, tracker.avg_rewards, metrics_history
    _save_artifacts(artifacts_dir, checkpoint_dir, experiment_name, metrics_history,
                    training_episodes, episode_rewards, tracker.eval_episodes, tracker.rewards,
                    tracker.avg_rewards, target_reward, total_steps, logger, exp_prefix)
    return tracker.rewards, tracker.avg_rewards, metrics_history


def _log_episode(logger, prefix, episode_num, ep_reward, episode_rewards, log_interval,
                 total_steps, start_time):
    if episode_num % log_interval == 0:
        logger.info("%s episode=%d reward=%.2f avg_reward=%.2f steps=%d time=%.2fs", prefix,
                    episode_num, ep_reward, np.mean(episode_rewards[-log_interval:]), total_steps,
                    time.time() - start_time)


def _train_single(env, agent, max_episodes, log_interval, eval_interval, steps_per_update,
                  exp_seed, logger, prefix, mh, tracker, start_time):
    """The reference loop (routine.py:121-243) on the one-env facade."""
    episode_rewards, training_episodes = [], []
    total_steps = episode_num = 0
    done, flat_state = True, None
    while episode_num < max_episodes:
        steps_collected = 0
        t_update = time.time()
        while steps_collected < steps_per_update and episode_num < max_episodes:
            episode_num += 1
            state, _ = env.reset(seed=exp_seed + episode_num)
            flat_state = state.reshape(-1)
            ep_reward, done = 0.0, False
            while not done and steps_collected < steps_per_update:
                action, pre_tanh, log_prob, value = agent.select_action(flat_state)
                nxt, reward, terminated, truncated, _ = env.step(action)
                done = terminated or truncated
                flat_next = nxt.reshape(-1)
                agent.memory.store(flat_state, action, pre_tanh, reward, flat_next, log_prob, done, value)
                flat_state = flat_next
                ep_reward += reward
                steps_collected += 1
                total_steps += 1
            episode_rewards.append(ep_reward)
            training_episodes.append(episode_num)
            mh["episode_rewards"].append(ep_reward)
            mh["episode_numbers"].append(episode_num)
            _log_episode(logger, prefix, episode_num, ep_reward, episode_rewards, log_interval,
                         total_steps, start_time)
            if episode_num % eval_interval == 0:
                tracker.on_episode(episode_num)
        final_value = 0.0
        if not done:
            with torch.no_grad():
                _, _, v = agent.actor_critic.forward(flat_state)
                final_value = float(v.cpu().item())
        upd = agent.update(last_value=final_value)
        mh["policy_updates"].append({"episode": episode_num, "steps": steps_collected,
                                     "time": time.time() - t_update, **upd})
    return episode_rewards, training_episodes, total_steps


def _train_vector(env, agent, max_episodes, log_interval, eval_interval, steps_per_update,
                  exp_seed, logger, prefix, mh, tracker, start_time):
    """E lockstep envs, device rollout of T steps, batched PPO update.

    With a process group on the agent (one rank per GPU, envs env_offset = rank*E of world*E),
    every rank steps its own E envs and joins the update's collectives; the episode stream is
    gathered so all ranks count the same episodes and stop after the same update, and rank 0
    alone evaluates and writes artifacts."""
    from ppo.agent import RolloutBuffer
    from ppo.rollout import LockstepRollout

    group = getattr(agent, "_dist", None)
    rank, world = _rank_world(group)
    base = env.unwrapped
    E = base.num_envs
    sd = _flat_dim(env)
    T = max(1, math.ceil(steps_per_update / E))
    buf = RolloutBuffer(T, E, sd, 2, base.device)
    base.set_seed_schedule(exp_seed)
    obs, _ = env.reset()
    buf.states[0].copy_(obs.reshape(E, sd))
    roll = LockstepRollout(agent, base, buf, use_graph=getattr(agent, "use_graphs", True))
    episode_rewards, training_episodes = [], []
    total_steps = episode_num = 0
    while episode_num < max_episodes:
        t_update = time.time()
        roll.run()
        total_steps += T * E * world
        upd = agent.update_rollout(buf, agent.value(buf.states[T]))
        # episode bookkeeping, in (step, global env) order -- identical on every rank
        for r in _episode_ends(buf.dones, buf.ep_return, group):
            if episode_num >= max_episodes:
                break
            episode_num += 1
            r = float(r)
            episode_rewards.append(r)
            training_episodes.append(episode_num)
            mh["episode_rewards"].append(r)
            mh["episode_numbers"].append(episode_num)
            _log_episode(logger, prefix, episode_num, r, episode_rewards, log_interval,
                         total_steps, start_time)
            if episode_num % eval_interval == 0 and rank == 0:
                tracker.on_episode(episode_num)
        mh["policy_updates"].append({"episode": episode_num, "steps": T * E * world,
                                     "time": time.time() - t_update, **upd})
        buf.states[0].copy_(buf.states[T])
    return episode_rewards, training_episodes, total_steps


def train_group(group, experiment_names, exp_seeds, max_episodes=500, target_reward=0.0,
                log_interval=20, eval_interval=50, loggers=None):
    """train_with_experiment_name for every experiment of an ExperimentGroup (ppo/group.py) at
    once: one grouped rollout + update per iteration, then each experiment's bookkeeping exactly
    as _train_vector does it on its own [T, E] slice (episode stream in (step, env) order,
    evaluation every ``eval_interval`` episodes on its own eval envs, best / solved checkpoints,
    artifacts).  An experiment that reaches ``max_episodes`` stops where its solo run stops; the
    group keeps stepping it (its later state is never read) until every experiment is done.
    Returns, per experiment, the reference's (rewards, avg_rewards, metrics_history), each equal
    to its solo run's: the group's experiments are bit-identical to solo runs
    (tests/test_group_gpu.py) and evaluation draws no random numbers."""
    return train_batch(group, [group], experiment_names, exp_seeds, max_episodes=max_episodes,
                       target_reward=target_reward, log_interval=log_interval,
                       eval_interval=eval_interval, loggers=loggers)


def train_batch(stepper, groups, experiment_names, exp_seeds, max_episodes=500, target_reward=0.0,
                log_interval=20, eval_interval=50, loggers=None):
    """train_group over the experiments of several ExperimentGroups stepped together: `stepper`
    is the ExperimentGroup itself (groups = [it]) or a GroupBatch over `groups` (ppo/group.py:
    the cells of one hidden width in one set of launches).  experiment_names / exp_seeds /
    loggers list every group's experiments in group order; each experiment's bookkeeping is its
    solo run's, on its own [T, E] slice of its group's rollout."""
    members = [(g, j) for g in groups for j in range(g.G)]
    if len(experiment_names) != len(members) or len(exp_seeds) != len(members):
        raise ValueError(f"train_batch: {len(members)} experiments, "
                         f"{len(experiment_names)} names, {len(exp_seeds)} seeds")
    artifacts_dir = ensure_artifacts_dir()
    checkpoint_dir = os.path.join(artifacts_dir, "checkpoints")
    os.makedirs(checkpoint_dir, exist_ok=True)
    start_time = time.time()
    runs = []
    for k, (grp, j) in enumerate(members):
        name = experiment_names[k]
        logger = loggers[k] if loggers else setup_experiment_logger(name)
        prefix = f"[{name}]" if name else ""
        logger.info(f"{prefix} Starting training for experiment: {name} (group of {grp.G}, "
                    f"batch of {len(members)})")
        mh = {"experiment_name": name, "episode_rewards": [], "eval_rewards": [],
              "avg_eval_rewards": [], "policy_updates": [], "episode_numbers": [],
              "eval_episode_numbers": [], "timestamps": []}
        tracker = _EvalTracker(grp.solo_envs[j], grp.agents[j], int(exp_seeds[k]),
                               target_reward, checkpoint_dir, name, mh, logger, prefix, start_time)
        logger.info(f"{prefix} Performing initial evaluation...")
        runs.append({"name": name, "logger": logger, "prefix": prefix, "mh": mh,
                     "tracker": tracker, "episode_rewards": [], "training_episodes": [],
                     "episode_num": 0, "total_steps": 0, "done": max_episodes <= 0,
                     "group": grp, "j": j, "pending": []})
    # every experiment's evaluations run together (evaluate_many: the same results as one
    # evaluate each -- deterministic episodes, no random numbers drawn)
    first = evaluate_many([(r["tracker"].env, r["tracker"].agent, r["tracker"].exp_seed)
                           for r in runs])
    for r, v in zip(runs, first):
        r["tracker"].initial(v)
    while not all(r["done"] for r in runs):
        t_update = time.time()
        stepper.rollout()
        upds = stepper.update(return_metrics=True)
        if len(groups) > 1 or stepper is not groups[0]:  # a GroupBatch: one list per group
            upds = [m for per_group in upds for m in per_group]
        for r, upd in zip(runs, upds):
            if r["done"]:
                continue
            grp, j = r["group"], r["j"]
            E, T = grp.E, grp.T
            r["total_steps"] += T * E
            sl = slice(j * E, (j + 1) * E)
            for ret in _episode_ends(grp.buf.dones[:, sl], grp.buf.ep_return[:, sl]):
                if r["episode_num"] >= max_episodes:
                    break
                r["episode_num"] += 1
                ret = float(ret)
                r["episode_rewards"].append(ret)
                r["training_episodes"].append(r["episode_num"])
                r["mh"]["episode_rewards"].append(ret)
                r["mh"]["episode_numbers"].append(r["episode_num"])
                _log_episode(r["logger"], r["prefix"], r["episode_num"], ret, r["episode_rewards"],
                             log_interval, r["total_steps"], start_time)
                if r["episode_num"] % eval_interval == 0:
                    r["pending"].append(r["episode_num"])
            r["mh"]["policy_updates"].append({"episode": r["episode_num"], "steps": T * E,
                                              "time": time.time() - t_update, **upd})
            if r["episode_num"] >= max_episodes:
                r["done"] = True
        # this iteration's evaluations (weights unchanged since its update): one per experiment
        # that crossed an evaluation point, all together; a second point in the same iteration
        # evaluates the same weights and gets the same (memoised) value
        due = [r for r in runs if r["pending"]]
        if due:
            vals = evaluate_many([(r["tracker"].env, r["tracker"].agent, r["tracker"].exp_seed)
                                  for r in due])
            for r, v in zip(due, vals):
                for ep in r["pending"]:
                    r["tracker"].on_episode(ep, v)
                r["pending"] = []
    out = []
    for r in runs:
        tr = r["tracker"]
        _save_artifacts(artifacts_dir, checkpoint_dir, r["name"], r["mh"], r["training_episodes"],
                        r["episode_rewards"], tr.eval_episodes, tr.rewards, tr.avg_rewards,
                        target_reward, r["total_steps"], r["logger"], r["prefix"])
        out.append((tr.rewards, tr.avg_rewards, r["mh"]))
    return out


def _rank_world(group):
    if group is None:
        return 0, 1
    return torch.distributed.get_rank(group), torch.distributed.get_world_size(group)


def _episode_ends(dones, rets, group=None):
    """Returns of the episodes that ended in a [T, E] rollout, in (step, env) order.

    Over a process group each rank's [T, E] slice is all-gathered and laid side by side, so
    every rank sees the [T, world*E] stream one process stepping all world*E envs (rank r's at
    r*E..) would, and counts the same episodes in the same order."""
    pack = torch.stack([dones.to(torch.float64), rets.to(torch.float64)])
    if group is not None:
        if torch.distributed.get_backend(group) == "gloo":
            pack = pack.cpu()
        parts = [torch.empty_like(pack) for _ in range(torch.distributed.get_world_size(group))]
        torch.distributed.all_gather(parts, pack.contiguous(), group=group)
        pack = torch.cat(parts, dim=2)
    pack = pack.cpu().numpy()
    return pack[1][pack[0] != 0]
