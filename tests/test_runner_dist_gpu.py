"""One experiment across ranks through ExperimentRunner: two ranks on one GPU
with gloo standing in for RCCL, as torchrun would launch them (WORLD_SIZE / RANK / LOCAL_RANK in
the env).  The ranks must count the same episodes, run the same number of updates, end with
identical weights, and only rank 0 evaluates and writes artifacts."""

import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
E, EPISODES = 64, 160


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "highway-rope-ppo_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      LOCAL_RANK=str(rank), WORLD_SIZE=str(world), HWY_DIST_BACKEND="gloo")
    os.chdir(os.path.join(out_dir, f"cwd{rank}"))
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition, ConditionHP, Experiment
    from experiments.runner import ExperimentRunner

    hp = ConditionHP(lr=3e-4, clip_eps=0.2, epochs=2, batch_size=64, hidden_dim=64)
    hp.steps_per_update = E * 8
    exp = Experiment(name="dist_runner", condition=Condition.SORTED, hp=hp, seed=42,
                     max_episodes=EPISODES, target_reward=1e9,
                     extra={"num_envs": E, "eval_interval": 50, "num_minibatches": 4})
    runner = ExperimentRunner(HIGHWAY_CONFIG)
    agent_box = {}
    make = runner._create_agent

    def _keep(*a, **k):
        agent_box["a"] = make(*a, **k)
        return agent_box["a"]

    runner._create_agent = _keep
    res = runner.launch(exp)
    mh = res.get("metrics_history", {})
    w = torch.cat([p.detach().reshape(-1).cpu() for p in agent_box["a"].actor_critic.parameters()])
    out = {"status": res["status"], "error": res.get("error_message"), "rank": res.get("rank", 0),
           "episodes": mh.get("episode_numbers", []), "updates": len(mh.get("policy_updates", [])),
           "evals": len(res.get("rewards", [])), "wsum": float(w.double().sum()),
           "wabs": float(w.double().abs().sum()),
           "gen_seed": int(agent_box["a"].generator.initial_seed())}
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    torch.distributed.destroy_process_group()


def test_runner_one_experiment_over_two_ranks(tmp_path):
    for r in range(2):
        (tmp_path / f"cwd{r}").mkdir()
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    r0 = json.loads((tmp_path / "rank0.json").read_text())
    r1 = json.loads((tmp_path / "rank1.json").read_text())
    assert r0["status"] == r1["status"] == "COMPLETED", (r0["error"], r1["error"])
    assert r0["rank"] == 0 and r1["rank"] == 1
    assert r0["episodes"] == r1["episodes"] == list(range(1, EPISODES + 1))
    assert r0["updates"] == r1["updates"] >= 1
    assert r0["wsum"] == r1["wsum"] and r0["wabs"] == r1["wabs"]  # replicas identical
    # each rank samples its envs' exploration noise from its own stream (the same
    # stream on every rank would give global env r*E+e the noise of env e)
    assert r0["gen_seed"] != r1["gen_seed"]
    assert r0["evals"] == 1 + EPISODES // 50 and r1["evals"] == 0
    assert (tmp_path / "cwd0/artifacts/highway-ppo/summary_dist_runner.csv").exists()
    assert not (tmp_path / "cwd1/artifacts/highway-ppo/summary_dist_runner.csv").exists()
