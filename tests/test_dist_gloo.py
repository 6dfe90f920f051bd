"""Env-sharded data parallelism on CPU with gloo, world sizes 2 and 4.

Each rank owns its own slice of samples; per optimizer step the flat gradient bucket is
all-reduced (mean), and advantage statistics are reduced once per update.  The sharded result
must equal one process running the same update on the concatenated data with global
minibatch i = rank0's minibatch i ++ rank1's minibatch i ++ ... (world 4 rehearses more ranks
than the one-GPU box can run)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

SD, H, EPOCHS, NMB, NLOC = 12, 16, 3, 4, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(rank, n=NLOC):
    g = np.random.default_rng(100 + rank)
    return dict(
        s=torch.as_tensor(g.normal(size=(n, SD)).astype(np.float32)),
        z=torch.as_tensor(g.normal(size=(n, 2)).astype(np.float32) * 0.5),
        lp=torch.as_tensor(g.normal(size=n).astype(np.float32) - 2.0),
        a=torch.as_tensor(g.normal(size=n).astype(np.float32)),
        r=torch.as_tensor(g.normal(size=n).astype(np.float32)),
        perm=torch.as_tensor(g.permutation(n)),
    )


def _make_agent(group=None):
    import sys

    from ppo.agent import PPOAgent

    torch.manual_seed(7)
    return PPOAgent(SD, 2, lr=1e-3, epochs=EPOCHS, batch_size=16, hidden_dim=H,
                    device=torch.device("cpu"), num_minibatches=NMB, use_graphs=False,
                    process_group=group)


def _worker(rank, world, port, out_dir):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "highway-rope-ppo_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    if rank > 0:
        torch.manual_seed(999 + rank)  # different local init: the broadcast must make weights equal
    agent = _make_agent(torch.distributed.group.WORLD)
    d = _data(rank)
    adv_n = agent.normalize_advantages(d["a"])
    mb = NLOC // NMB
    batches = [d["perm"][i * mb:(i + 1) * mb] for i in range(NMB)]
    agent._run_epochs(d["s"], d["z"], d["lp"], adv_n, d["r"], batches)
    torch.save({"state": agent.actor_critic.state_dict(), "adv": adv_n},
               os.path.join(out_dir, f"rank{rank}.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_update_equals_single_process(tmp_path, world):
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    rs = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    # replicas stay identical
    for r in rs[1:]:
        for k in rs[0]["state"]:
            torch.testing.assert_close(rs[0]["state"][k], r["state"][k], rtol=0, atol=0)
    # single process on the concatenated data
    ds = [_data(r) for r in range(world)]
    cat = {k: torch.cat([d[k] for d in ds]) for k in ("s", "z", "lp", "a", "r")}
    a = cat["a"]
    adv_n = (a - a.mean()) / (a.std() + 1e-8)
    torch.testing.assert_close(torch.cat([r["adv"] for r in rs]), adv_n, rtol=1e-5, atol=1e-6)
    agent = _make_agent(None)
    mb = NLOC // NMB
    batches = [torch.cat([d["perm"][i * mb:(i + 1) * mb] + r * NLOC for r, d in enumerate(ds)])
               for i in range(NMB)]
    agent._run_epochs(cat["s"], cat["z"], cat["lp"], adv_n, cat["r"], batches)
    for k, v in agent.actor_critic.state_dict().items():
        torch.testing.assert_close(rs[0]["state"][k], v, rtol=2e-5, atol=2e-6, msg=k)


# ---- the runner's episode stream over ranks (training/routine.py _episode_ends) ----
T_EP, E_EP = 5, 6


def _episode_slice(rank):
    g = np.random.default_rng(300 + rank)
    dones = torch.as_tensor(g.random((T_EP, E_EP)) < 0.3)
    rets = torch.as_tensor(g.normal(size=(T_EP, E_EP)).astype(np.float32) * 10)
    return dones, rets


def _episode_worker(rank, world, port, out_dir):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "highway-rope-ppo_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from training.routine import _episode_ends

    ends = _episode_ends(*_episode_slice(rank), torch.distributed.group.WORLD)
    np.save(os.path.join(out_dir, f"ends{rank}.npy"), ends)
    torch.distributed.destroy_process_group()


def test_episode_ends_single_process_order():
    from training.routine import _episode_ends

    dones, rets = _episode_slice(0)
    want = [float(rets[t, e]) for t in range(T_EP) for e in range(E_EP) if dones[t, e]]
    np.testing.assert_array_equal(_episode_ends(dones, rets), np.array(want))


def test_episode_ends_gathered_over_ranks_in_global_env_order(tmp_path):
    """Every rank counts the episodes of one process stepping both ranks' envs side by side
    (rank r's envs at r*E..), so all ranks stop after the same update."""
    port = _free_port()
    mp.start_processes(_episode_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    (d0, r0), (d1, r1) = _episode_slice(0), _episode_slice(1)
    dones, rets = torch.cat([d0, d1], 1), torch.cat([r0, r1], 1)
    want = [float(rets[t, e]) for t in range(T_EP) for e in range(2 * E_EP) if dones[t, e]]
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"ends{r}.npy"), np.array(want))
