"""evaluate() one experiment at a time against evaluate_many() (training/routine.py) on the same
(env, agent, seed) items -- development aid: prints both results per item."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "highway-rope-ppo_amd"))
import torch  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from ppo.agent import PPOAgent
    from ppo.group import build_group
    from training import routine

    cond = Condition[sys.argv[1]] if len(sys.argv) > 1 else Condition.SHUFFLED_RANKPE
    d = None if cond is Condition.SORTED else 4
    seeds = [42, 1042, 7]
    grp = build_group(cond, HIGHWAY_CONFIG, seeds, 16, 32, DEV,
                      lambda sd: PPOAgent(sd, 2, device=DEV, lr=3e-4, epochs=2, batch_size=64,
                                          hidden_dim=256), d_embed=d)
    items = [(grp.solo_envs[j], grp.agents[j], s) for j, s in enumerate(seeds)]

    def clear():
        for env, _, _ in items:
            env.unwrapped._eval_memo = None

    seq = []
    for what in ("solo", "solo", "many", "many", "solo"):
        clear()
        seq.append((what, routine.evaluate_many(items) if what == "many"
                    else [routine.evaluate(e, a, num_episodes=5, exp_seed=s) for e, a, s in items]))
    for what, v in seq:
        print(cond.name, what, v, flush=True)


if __name__ == "__main__":
    main()


def detail():
    """First step of item 0, solo against grouped: the actions and the next observations."""
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from hwy.ppo_native import GroupAct, fused_act
    from hwy.vec_env import GroupEnvStep
    from ppo.agent import PPOAgent
    from ppo.group import build_group
    from training.routine import _eval_env_like

    seeds = [42, 1042]
    grp = build_group(Condition.SORTED, HIGHWAY_CONFIG, seeds, 16, 32, DEV,
                      lambda sd: PPOAgent(sd, 2, device=DEV, lr=3e-4, epochs=2, batch_size=64,
                                          hidden_dim=256))
    evs = [_eval_env_like(grp.solo_envs[j], 5) for j in range(2)]
    ev_solo = _eval_env_like(grp.solo_envs[0], 5)
    sd = torch.arange(5, device=DEV, dtype=torch.int64) + 1042
    o_solo, _ = ev_solo.reset(seeds=sd)
    obs = [evs[j].reset(seeds=torch.arange(5, device=DEV, dtype=torch.int64) + s + 1000)[0]
           for j, s in enumerate(seeds)]
    torch.cuda.synchronize()
    print("reset obs equal", torch.equal(o_solo, obs[0]), o_solo.data_ptr() == ev_solo.obs_buf.data_ptr(),
          obs[0].shape, flush=True)
    a_solo = fused_act(grp.agents[0], o_solo.reshape(5, -1), True)[0].clone()
    act = GroupAct(grp.agents, 5)
    tiles = act.tiles()
    outs = [[torch.empty(5, 2, device=DEV), torch.empty(5, 2, device=DEV), torch.empty(5, device=DEV),
             torch.empty(5, device=DEV)] for _ in range(2)]
    rows = [(obs[j].data_ptr(), None) + tuple(t.data_ptr() for t in outs[j]) for j in range(2)]
    act.launch(rows, tiles)
    torch.cuda.synchronize()
    print("tiles", [t is not None for t in tiles], "actions equal", torch.equal(a_solo, outs[0][0]),
          a_solo[:2].tolist(), outs[0][0][:2].tolist(), flush=True)
    r = torch.empty(10, device=DEV)
    te = torch.empty(10, dtype=torch.uint8, device=DEV)
    tr = torch.empty(10, dtype=torch.uint8, device=DEV)
    GroupEnvStep(evs).launch([(outs[j][0], obs[j], r[5 * j:5 * j + 5], te[5 * j:5 * j + 5],
                               tr[5 * j:5 * j + 5], None, None) for j in range(2)])
    o2, r2, te2, tr2, _ = ev_solo.step(a_solo.contiguous())
    torch.cuda.synchronize()
    print("step: obs equal", torch.equal(o2, obs[0]), "rew", r2.tolist(), r[:5].tolist(),
          "te", te2.tolist(), te[:5].tolist(), flush=True)


if __name__ == "__main__" and os.environ.get("DETAIL"):
    detail()


def detail2():
    """Solo and grouped evaluation loops side by side, item by item: the first step at which an
    observation, reward or flag differs."""
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from hwy.ppo_native import GroupAct, fused_act
    from hwy.vec_env import GroupEnvStep
    from ppo.agent import PPOAgent
    from ppo.group import build_group
    from training.routine import _eval_env_like

    seeds = [42, 1042, 7]
    n = 5
    grp = build_group(Condition.SORTED, HIGHWAY_CONFIG, seeds, 16, 32, DEV,
                      lambda sd: PPOAgent(sd, 2, device=DEV, lr=3e-4, epochs=2, batch_size=64,
                                          hidden_dim=256))
    k = len(seeds)
    evs = [_eval_env_like(grp.solo_envs[j], n) for j in range(k)]
    solos = [_eval_env_like(grp.solo_envs[j], n) for j in range(k)]
    obs = [evs[j].reset(seeds=torch.arange(n, device=DEV, dtype=torch.int64) + s + 1000)[0]
           for j, s in enumerate(seeds)]
    sobs = [solos[j].reset(seeds=torch.arange(n, device=DEV, dtype=torch.int64) + s + 1000)[0]
            for j, s in enumerate(seeds)]
    act = GroupAct(grp.agents, n)
    tiles = act.tiles()
    outs = [[torch.empty(n, 2, device=DEV), torch.empty(n, 2, device=DEV),
             torch.empty(n, device=DEV), torch.empty(n, device=DEV)] for _ in range(k)]
    rows = [(obs[j].data_ptr(), None) + tuple(t.data_ptr() for t in outs[j]) for j in range(k)]
    rew = torch.empty(k * n, device=DEV)
    te = torch.empty(k * n, dtype=torch.uint8, device=DEV)
    tr = torch.empty(k * n, dtype=torch.uint8, device=DEV)
    ios = [(outs[j][0], obs[j], rew[j * n:(j + 1) * n], te[j * n:(j + 1) * n],
            tr[j * n:(j + 1) * n], None, None) for j in range(k)]
    step = GroupEnvStep(evs)
    for t in range(60):
        act.launch(rows, tiles)
        step.launch(ios)
        for j in range(k):
            a = fused_act(grp.agents[j], sobs[j].reshape(n, -1), True)[0]
            o2, r2, te2, tr2, _ = solos[j].step(a.contiguous())
            torch.cuda.synchronize()
            ok = (torch.equal(a, outs[j][0]), torch.equal(o2, obs[j]),
                  torch.equal(r2, rew[j * n:(j + 1) * n]), torch.equal(te2, te[j * n:(j + 1) * n]))
            if not all(ok):
                print("first mismatch step", t, "item", j, "act/obs/rew/te", ok, flush=True)
                return
    print("60 steps equal", flush=True)


if __name__ == "__main__" and os.environ.get("DETAIL2"):
    detail2()


def detail3():
    """routine._run_eval_group against routine._run_eval_vector item by item, fresh eval envs."""
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from ppo.agent import PPOAgent
    from ppo.group import build_group
    from training import routine

    seeds = [42, 1042, 7]
    grp = build_group(Condition.SORTED, HIGHWAY_CONFIG, seeds, 16, 32, DEV,
                      lambda sd: PPOAgent(sd, 2, device=DEV, lr=3e-4, epochs=2, batch_size=64,
                                          hidden_dim=256))
    items = [(grp.solo_envs[j], grp.agents[j], s) for j, s in enumerate(seeds)]
    g = routine._run_eval_group(items, 5)
    v = [routine._run_eval_vector(e, a, 5, s) for e, a, s in items]
    g2 = routine._run_eval_group(items, 5)
    g1 = [routine._run_eval_group([it], 5)[0] for it in items]
    print("group", g, "\nvector", v, "\ngroup again", g2, "\ngroup of one", g1, flush=True)


if __name__ == "__main__" and os.environ.get("DETAIL3"):
    detail3()
