"""ExperimentGroup (ppo/group.py): G experiments of one condition batched into the launches
themselves (grouped env handle, grouped acting, grouped minibatch steps) must each be bit for
bit their solo run -- the runner's construction (experiments/runner.py:102-138) and
training/routine.py's _train_vector loop (LockstepRollout + update_rollout) with the same seed.
Checked on every rollout row, the final weights, Adam moments and the metrics."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _hp(H, epochs=2):
    return dict(lr=3e-4, epochs=epochs, batch_size=64, hidden_dim=H)


def _solo(cond, d, seed, E, T, iters, H, overrides):
    from config.base_config import HIGHWAY_CONFIG
    from experiments.wrappers import make_env
    from ppo.agent import PPOAgent, RolloutBuffer
    from ppo.rollout import LockstepRollout
    from utils.reproducibility import set_random_seeds

    set_random_seeds(seed)
    env = make_env(cond, HIGHWAY_CONFIG, d_embed=d,
                   env_overrides=dict(overrides, num_envs=E, device=DEV, autoreset=True))
    if hasattr(env, "to"):
        env = env.to(DEV)
    base = env.unwrapped
    sd = base.obs_rows * base.obs_features
    agent = PPOAgent(sd, 2, device=DEV, **_hp(H))
    base.set_seed_schedule(seed)
    obs, _ = env.reset()
    buf = RolloutBuffer(T, E, sd, 2, DEV)
    buf.states[0].copy_(obs.reshape(E, sd))
    roll = LockstepRollout(agent, base, buf)
    hist, metrics = [], []
    for _ in range(iters):
        roll.run()
        hist.append({k: getattr(buf, k).clone() for k in ("states", "actions", "rewards", "dones",
                                                          "log_probs", "values")})
        metrics.append(agent.update_rollout(buf, agent.value(buf.states[T])))
        buf.states[0].copy_(buf.states[T])
    torch.cuda.synchronize()
    return agent, hist, metrics, env


@pytest.mark.parametrize("cond_name,d,H,order", [("SORTED", None, 256, None),
                                                 ("SHUFFLED_RANKPE", 4, 384, "shuffled"),
                                                 ("SHUFFLED_ROPE", 4, 256, "shuffled")])
def test_group_matches_solo_runs_bit_for_bit(cond_name, d, H, order):
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from ppo.group import build_group

    cond = Condition[cond_name]
    seeds, E, T, iters = [42, 1042, 2042], 16, 16, 3
    overrides = {} if order is None else {"observation": {"order": order}}
    from ppo.agent import PPOAgent

    grp = build_group(cond, HIGHWAY_CONFIG, seeds, E, T, DEV,
                      lambda sd: PPOAgent(sd, 2, device=DEV, **_hp(H)), d_embed=d,
                      env_overrides=overrides)
    ghist, gmet = [], []
    for _ in range(iters):
        grp.rollout()
        b = grp.buf
        ghist.append({k: getattr(b, k).clone() for k in ("states", "actions", "rewards", "dones",
                                                         "log_probs", "values")})
        gmet.append(grp.update())
    torch.cuda.synchronize()
    assert grp.agents[0]._fused is not None and grp.agents[0]._fused.mb == 64
    for g, s in enumerate(seeds):
        agent, hist, metrics, env = _solo(cond, d, s, E, T, iters, H, overrides)
        sl = slice(g * E, (g + 1) * E)
        for it in range(iters):
            for k, v in hist[it].items():
                assert torch.equal(ghist[it][k][:, sl], v), (g, it, k)
            assert gmet[it][g] == metrics[it], (g, it)
        for (k, va), (_, vb) in zip(agent.actor_critic.state_dict().items(),
                                    grp.agents[g].actor_critic.state_dict().items()):
            assert torch.equal(va, vb), (g, k)
        Fs, Fg = agent._fused, grp.agents[g]._fused
        assert torch.equal(Fs.m, Fg.m) and torch.equal(Fs.v, Fg.v), g
        assert int(Fs.counters[0]) == int(Fg.counters[0]) == iters * 2 * (T * E // 64)
        env.close()
    # the episodes of each experiment come out of its own slice
    assert grp.episode_returns(0).numel() == int(grp.buf.dones[:, :E].sum())


def test_group_batch_of_cells_with_different_state_dims_matches_solo_runs():
    """GroupBatch: two h256 cells whose learners differ in state dim (sorted, S 60; shuffled
    RankPE d_embed 4, S 120) stepped as one set of launches -- one acting launch per step over
    both cells' learners, one grouped minibatch step whose grids cover the larger learner --
    and every experiment still equals its solo run bit for bit."""
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from ppo.agent import PPOAgent
    from ppo.group import GroupBatch, build_group

    E, T, iters = 16, 16, 3
    cells = [(Condition.SORTED, None, [42, 1042]), (Condition.SHUFFLED_RANKPE, 4, [7, 2042, 99])]
    groups = [build_group(c, HIGHWAY_CONFIG, seeds, E, T, DEV,
                          lambda sd: PPOAgent(sd, 2, device=DEV, **_hp(256)), d_embed=d)
              for c, d, seeds in cells]
    assert {g.sd for g in groups} == {60, 120}
    batch = GroupBatch(groups)
    hist = []
    for _ in range(iters):
        batch.rollout()
        hist.append([{k: getattr(g.buf, k).clone() for k in ("states", "rewards", "log_probs")}
                     for g in groups])
        batch.update()
    torch.cuda.synchronize()
    for gi, (c, d, seeds) in enumerate(cells):
        for j, s in enumerate(seeds):
            agent, shist, _, env = _solo(c, d, s, E, T, iters, 256, {})
            sl = slice(j * E, (j + 1) * E)
            for it in range(iters):
                for k, v in hist[it][gi].items():
                    assert torch.equal(v[:, sl], shist[it][k]), (gi, j, it, k)
            for (k, va), (_, vb) in zip(agent.actor_critic.state_dict().items(),
                                        groups[gi].agents[j].actor_critic.state_dict().items()):
                assert torch.equal(va, vb), (gi, j, k)
            env.close()
    # one argument-table preparation for the whole batch; the third rollout (the second at the
    # updated weights' tile images) was captured as a graph
    assert batch.stats["update_prepare"] == 1 and batch.stats["rollout_capture"] == 1


def test_group_env_seeds_follow_each_experiments_schedule():
    """hwy_set_seed_groups: group g's envs reset with seed_bases[g] + l + 1 (+ E per episode),
    so a grouped handle's first observations equal each solo handle's."""
    from config.base_config import HIGHWAY_CONFIG
    from hwy.vec_env import HighwayVecEnv

    E, seeds = 8, [5, 900, 77]
    grp = HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E * len(seeds), device=DEV)
    grp.set_seed_groups(seeds, E)
    obs, _ = grp.reset()
    obs = obs.clone()
    for g, s in enumerate(seeds):
        solo = HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device=DEV)
        solo.set_seed_schedule(s)
        o, _ = solo.reset()
        assert torch.equal(obs[g * E:(g + 1) * E], o), g
        solo.close()
    with pytest.raises(Exception):
        grp.set_seed_groups(seeds[:2], E)  # 2 x 8 envs do not cover 24
    grp.close()


def test_runner_launch_group_equals_launch(tmp_path, monkeypatch):
    """ExperimentRunner.launch_group (one ExperimentGroup for a cell's seeds) returns, per
    experiment, exactly what launch() returns for it alone: the episode stream, every
    evaluation and the moving averages (training/routine.py:train_group vs _train_vector)."""
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition, ConditionHP, Experiment
    from experiments.runner import ExperimentRunner

    monkeypatch.chdir(tmp_path)

    def exp(seed):
        hp = ConditionHP(lr=3e-4, clip_eps=0.2, epochs=2, batch_size=64, hidden_dim=256,
                         d_embed=4)
        hp.entropy_coef = 0.005
        hp.steps_per_update = 16 * 32
        return Experiment(name=f"grp_rank_seed{seed}", condition=Condition.SHUFFLED_RANKPE,
                          hp=hp, seed=seed, max_episodes=24, target_reward=1e9,
                          extra={"num_envs": 16, "num_minibatches": 8, "eval_interval": 8,
                                 "log_interval": 50}, env_config_overrides={})

    seeds = [42, 1042]
    grouped = ExperimentRunner(HIGHWAY_CONFIG).launch_group([exp(s) for s in seeds])
    for s, g in zip(seeds, grouped):
        solo = ExperimentRunner(HIGHWAY_CONFIG).launch(exp(s))
        assert solo["status"] == g["status"] == "COMPLETED", (solo.get("error_message"),
                                                              g.get("error_message"))
        assert g["rewards"] == solo["rewards"] and g["avg_rewards"] == solo["avg_rewards"], s
        mg, ms = g["metrics_history"], solo["metrics_history"]
        assert mg["episode_rewards"] == ms["episode_rewards"]
        assert mg["eval_episode_numbers"] == ms["eval_episode_numbers"]
        assert [u["loss"] for u in mg["policy_updates"]] == [u["loss"] for u in ms["policy_updates"]]
    assert (tmp_path / "artifacts").exists() or any(tmp_path.iterdir())


def test_group_eager_equals_graph_replay():
    """use_graphs=False (every rollout step and minibatch step launched eagerly) and the default
    graph capture / replay give the same experiments bit for bit."""
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from ppo.agent import PPOAgent
    from ppo.group import build_group

    E, T, iters, seeds = 16, 16, 3, [42, 1042]
    out = []
    for graphs in (True, False):
        grp = build_group(Condition.SHUFFLED_DISTPE, HIGHWAY_CONFIG, seeds, E, T, DEV,
                          lambda sd: PPOAgent(sd, 2, device=DEV, **_hp(256)), d_embed=4,
                          use_graphs=graphs)
        hist = []
        for _ in range(iters):
            grp.rollout()
            hist.append({k: getattr(grp.buf, k).clone() for k in ("states", "log_probs", "values")})
            hist[-1]["metrics"] = grp.update()
        torch.cuda.synchronize()
        w = [torch.cat([p.detach().reshape(-1) for p in ag.actor_critic.parameters()]).clone()
             for ag in grp.agents]
        out.append((hist, w, dict(grp.stats)))
        grp.close()
    (h1, w1, s1), (h0, w0, s0) = out
    for it in range(iters):
        for k in ("states", "log_probs", "values"):
            assert torch.equal(h1[it][k], h0[it][k]), (it, k)
        assert h1[it]["metrics"] == h0[it]["metrics"], it
    assert all(torch.equal(a, b) for a, b in zip(w1, w0))
    assert s1["rollout_capture"] >= 1 and s0.get("rollout_capture", 0) == 0


def test_grouped_env_step_equals_each_handles_own_step():
    """hwy_step_group: three handles that differ in env count, observation width, row order and
    fused wrapper (sorted / no PE, 8 envs; shuffled RoPE, 16; RankPE with seed groups, 3 x 8)
    stepped as ONE launch produce, step for step, exactly what each handle's own hwy_step
    produces: observations, rewards, flags and finished-episode returns and lengths, through
    crashes and in-kernel autoresets."""
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from experiments.wrappers import make_env
    from hwy.vec_env import GroupEnvStep
    from utils.reproducibility import set_random_seeds

    specs = [(Condition.SORTED, None, 8, {}, None),
             (Condition.SHUFFLED_ROPE, 4, 16, {"observation": {"order": "shuffled"}}, None),
             (Condition.SHUFFLED_RANKPE, 4, 24, {}, [5, 900, 77])]

    def make_set():
        envs = []
        for i, (cond, d, E, ov, groups) in enumerate(specs):
            set_random_seeds(1000 + i)  # RankPE draws its table from the global RNG
            env = make_env(cond, HIGHWAY_CONFIG, d_embed=d,
                           env_overrides=dict(ov, num_envs=E, device=DEV, autoreset=True))
            if hasattr(env, "to"):
                env = env.to(DEV)
            base = env.unwrapped
            if groups:
                base.set_seed_groups(groups, E // len(groups))
            else:
                base.set_seed_schedule(31 + i)
            env.reset()
            envs.append(base)
        return envs

    solo, grouped = make_set(), make_set()
    gstep = GroupEnvStep(grouped)

    def bufs(env):
        E = env.num_envs
        return (torch.empty(E, 2, device=DEV), torch.empty_like(env.obs_buf),
                torch.empty(E, device=DEV), torch.empty(E, dtype=torch.uint8, device=DEV),
                torch.empty(E, dtype=torch.uint8, device=DEV), torch.empty(E, device=DEV),
                torch.empty(E, dtype=torch.int32, device=DEV))

    bs, bg = [bufs(e) for e in solo], [bufs(e) for e in grouped]
    gen = torch.Generator(device=DEV).manual_seed(3)
    episodes = 0
    for step in range(60):
        for a, b in zip(bs, bg):
            a[0].copy_(torch.rand(a[0].shape, device=DEV, generator=gen) * 2 - 1)
            b[0].copy_(a[0])
        for env, a in zip(solo, bs):
            env.step_into(*a)
        gstep.launch(bg)
        torch.cuda.synchronize()
        for i, (a, b) in enumerate(zip(bs, bg)):
            for k in range(1, 7):
                assert torch.equal(a[k], b[k]), (step, i, k)
            episodes += int((a[3] | a[4]).sum())
    assert episodes > 0  # autoresets happened inside the compared window
    for env in solo + grouped:
        env.close()


def test_runner_launch_batch_equals_launch_group(tmp_path, monkeypatch):
    """ExperimentRunner.launch_batch (two h256 cells of different state dims stepped by one
    GroupBatch, training/routine.py:train_batch) returns, per experiment, exactly what
    launch_group returns for its cell alone."""
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition, ConditionHP, Experiment
    from experiments.runner import ExperimentRunner

    monkeypatch.chdir(tmp_path)

    def exp(cond, d, seed):
        hp = ConditionHP(lr=3e-4, clip_eps=0.2, epochs=2, batch_size=64, hidden_dim=256,
                         d_embed=d)
        hp.entropy_coef = 0.005
        hp.steps_per_update = 16 * 32
        return Experiment(name=f"b_{cond.name}_{seed}", condition=cond, hp=hp, seed=seed,
                          max_episodes=24, target_reward=1e9,
                          extra={"num_envs": 16, "num_minibatches": 8, "eval_interval": 8,
                                 "log_interval": 50}, env_config_overrides={})

    cells = [[exp(Condition.SORTED, None, s) for s in (42, 1042)],
             [exp(Condition.SHUFFLED_RANKPE, 4, s) for s in (7, 2042)]]
    batched = ExperimentRunner(HIGHWAY_CONFIG).launch_batch(cells)
    for cell, got in zip(cells, batched):
        alone = ExperimentRunner(HIGHWAY_CONFIG).launch_group(cell)
        for a, b in zip(alone, got):
            assert a["status"] == b["status"] == "COMPLETED", (a.get("error_message"),
                                                               b.get("error_message"))
            assert a["rewards"] == b["rewards"] and a["avg_rewards"] == b["avg_rewards"]
            ma, mb = a["metrics_history"], b["metrics_history"]
            assert ma["episode_rewards"] == mb["episode_rewards"]
            assert [u["loss"] for u in ma["policy_updates"]] == \
                [u["loss"] for u in mb["policy_updates"]]


@pytest.mark.parametrize("E", [4096, 16384])
def test_parameter_table_step_equals_hwy_step_at_rollout_sizes(E):
    """The lockstep rollout's env launch (hwy_step_group over its one handle: the launch
    parameters read from a device table) against hwy_step's by-value kernel on a twin handle, at
    the default line's 4,096 envs (4-wave build) and at 16,384 (6-wave build, more envs than
    four waves per SIMD): the same observations, rewards, flags and episode statistics."""
    from config.base_config import HIGHWAY_CONFIG
    from hwy.vec_env import GroupEnvStep, HighwayVecEnv

    envs = [HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device=DEV, autoreset=True, seed_base=42)
            for _ in range(2)]
    for env in envs:
        env.reset()

    def bufs():
        return (torch.empty(E, 2, device=DEV), torch.empty_like(envs[0].obs_buf),
                torch.empty(E, device=DEV), torch.empty(E, dtype=torch.uint8, device=DEV),
                torch.empty(E, dtype=torch.uint8, device=DEV), torch.empty(E, device=DEV),
                torch.empty(E, dtype=torch.int32, device=DEV))

    a, b = bufs(), bufs()
    g = GroupEnvStep([envs[1]])
    gen = torch.Generator(device=DEV).manual_seed(11)
    for step in range(24):
        a[0].copy_(torch.rand(E, 2, device=DEV, generator=gen) * 2 - 1)
        b[0].copy_(a[0])
        envs[0].step_into(*a)
        g.launch([b])
        torch.cuda.synchronize()
        for k in range(1, 7):
            assert torch.equal(a[k], b[k]), (step, k)
    for env in envs:
        env.close()
