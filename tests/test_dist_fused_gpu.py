"""The fused HIP update's data-parallel path (FusedPPO with a process group: graph(forward +
backward) -> all-reduce of the flat gradient -> graph(clip + Adam)) with 2 ranks on one GPU
(gloo carries the all-reduce; on a node the same code runs over RCCL).  The sharded update must
keep the replicas identical and equal one process on the concatenated minibatches."""

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
S, H, EPOCHS, NMB, NLOC = 60, 128, 2, 4, 1024


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(rank, dev):
    g = torch.Generator(device="cpu").manual_seed(100 + rank)
    d = dict(s=torch.randn(NLOC, S, generator=g), z=torch.randn(NLOC, 2, generator=g) * 0.5,
             lp=torch.randn(NLOC, generator=g) - 2.0, a=torch.randn(NLOC, generator=g),
             r=torch.randn(NLOC, generator=g), perm=torch.randperm(NLOC, generator=g))
    return {k: v.to(dev) for k, v in d.items()}


def _agent(dev, group=None):
    from ppo.agent import PPOAgent

    torch.manual_seed(7)
    return PPOAgent(S, 2, lr=3e-4, epochs=EPOCHS, hidden_dim=H, device=dev, num_minibatches=NMB,
                    use_graphs=True, process_group=group, backend="hip")


def _worker(rank, world, port, out_dir):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "highway-rope-ppo_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    if rank > 0:
        torch.manual_seed(999 + rank)  # different local init: the broadcast must make weights equal
    from hwy.ppo_native import FusedPPO

    agent = _agent(dev, torch.distributed.group.WORLD)
    d = _data(rank, dev)
    adv = agent.normalize_advantages(d["a"])
    F = FusedPPO(agent, NLOC // NMB, NMB, group=torch.distributed.group.WORLD, use_graphs=True)
    F.run(d["s"], d["z"].contiguous(), d["lp"], adv.contiguous(), d["r"], d["perm"])
    torch.cuda.synchronize()
    torch.save({"state": {k: v.cpu() for k, v in agent.actor_critic.state_dict().items()},
                "adv": adv.cpu()}, os.path.join(out_dir, f"rank{rank}.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_fused_sharded_update_equals_single_process(tmp_path, world):
    """world 4: four gloo ranks on the one GPU, rehearsing more ranks than the box has cards."""
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    rs = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    r0 = rs[0]
    for r in rs[1:]:  # replicas stay identical
        for k in r0["state"]:
            torch.testing.assert_close(r0["state"][k], r["state"][k], rtol=0, atol=0)
    from hwy.ppo_native import FusedPPO

    dev = torch.device("cuda", 0)
    ds = [_data(r, dev) for r in range(world)]
    cat = {k: torch.cat([d[k] for d in ds]) for k in ("s", "z", "lp", "a", "r")}
    adv = (cat["a"] - cat["a"].mean()) / (cat["a"].std() + 1e-8)
    torch.testing.assert_close(torch.cat([r["adv"] for r in rs]).to(dev), adv, rtol=1e-5,
                               atol=1e-6)
    mb = NLOC // NMB
    perm = torch.cat([torch.cat([d["perm"][i * mb:(i + 1) * mb] + r * NLOC
                                 for r, d in enumerate(ds)]) for i in range(NMB)])
    agent = _agent(dev)
    F = FusedPPO(agent, world * mb, NMB, use_graphs=True)
    F.run(cat["s"], cat["z"].contiguous(), cat["lp"], adv.contiguous(), cat["r"], perm.contiguous())
    torch.cuda.synchronize()
    steps = EPOCHS * NMB
    for k, v in agent.actor_critic.state_dict().items():
        dd = (r0["state"][k].to(dev) - v).abs()
        # Adam normalises each element's step, so fp32 noise in near-zero gradients can move an
        # element by up to ~lr per step: bound the worst case, require nearly all to agree
        assert dd.max().item() <= 2 * 3e-4 * steps, k
        assert (dd > 2e-5).float().mean().item() < 0.05, (k, dd.max().item())


def _rccl1_worker(rank, port, out_dir):
    """1-rank RCCL group: the epoch graph with the all-reduce captured, the per-step graphs with
    the all-reduce between them, and no process group must give the same weights."""
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "highway-rope-ppo_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from hwy.ppo_native import FusedPPO

    d = _data(0, dev)
    out = {}
    for tag, group, capture in (("captured", torch.distributed.group.WORLD, True),
                                ("stepwise", torch.distributed.group.WORLD, False),
                                ("local", None, False)):
        agent = _agent(dev, group)
        adv = agent.normalize_advantages(d["a"])
        F = FusedPPO(agent, NLOC // NMB, NMB, group=group, use_graphs=True)
        F.capture_collectives = capture
        for _ in range(2):  # the second update replays the captured graphs
            F.run(d["s"], d["z"].contiguous(), d["lp"], adv.contiguous(), d["r"], d["perm"])
        torch.cuda.synchronize()
        out[tag] = {"state": {k: v.cpu() for k, v in agent.actor_critic.state_dict().items()},
                    "captured": F._captured_collectives}
        # graphs holding RCCL collectives are freed while the communicator lives (the agent <->
        # FusedPPO cycle would otherwise free them after destroy_process_group: abort)
        F.release_graphs()
    torch.save(out, os.path.join(out_dir, "rccl1.pt"))
    torch.distributed.destroy_process_group()


def test_rccl_captured_allreduce_matches_stepwise_and_local(tmp_path):
    port = _free_port()
    mp.start_processes(_rccl1_worker, args=(port, str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    r = torch.load(tmp_path / "rccl1.pt", weights_only=True)
    assert r["captured"]["captured"] and not r["stepwise"]["captured"]
    for k in r["local"]["state"]:
        # the captured graph replays exactly what the per-step path launches
        torch.testing.assert_close(r["captured"]["state"][k], r["stepwise"]["state"][k], rtol=0,
                                   atol=0)
        # the group path recomputes clip_grad_norm_ from the reduced gradient (ppo_sumsq), whose
        # partial sums round differently from ppo_wsum's
        torch.testing.assert_close(r["captured"]["state"][k], r["local"]["state"][k], rtol=1e-4,
                                   atol=1e-6)


def _refusal_worker(rank, world, port, out_dir, refuse):
    """capture_collectives forced on over gloo; with `refuse` the first collective inside the
    capture raises (as a refused RCCL capture would), so FusedPPO must fall back to per-step
    graphs with the all-reduce between them."""
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "highway-rope-ppo_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    from hwy.ppo_native import FusedPPO

    group = torch.distributed.group.WORLD
    agent = _agent(dev, group)
    d = _data(rank, dev)
    adv = agent.normalize_advantages(d["a"])
    F = FusedPPO(agent, NLOC // NMB, NMB, group=group, use_graphs=True)
    tried = {"n": 0}
    if refuse:
        F.capture_collectives = True
        real = F._allreduce

        def _allreduce():
            if torch.cuda.is_current_stream_capturing():
                tried["n"] += 1
                raise RuntimeError("collective capture refused (test)")
            real()

        F._allreduce = _allreduce
    for _ in range(2):  # a second update replays the fallback graphs
        F.run(d["s"], d["z"].contiguous(), d["lp"], adv.contiguous(), d["r"], d["perm"])
    torch.cuda.synchronize()
    torch.save({"state": {k: v.cpu() for k, v in agent.actor_critic.state_dict().items()},
                "tried": tried["n"], "captured": F._captured_collectives,
                "capture_flag": F.capture_collectives},
               os.path.join(out_dir, f"{'refused' if refuse else 'plain'}{rank}.pt"))
    torch.distributed.destroy_process_group()


def test_refused_collective_capture_falls_back_to_per_step_graphs(tmp_path):
    """a refused capture of the epoch graph with its collectives falls back to
    per-step graphs with the all-reduce issued between them; the fallback's weights equal the
    HWY_GRAPH_COLLECTIVES=0 path's bit for bit on every rank."""
    for refuse in (False, True):
        mp.start_processes(_refusal_worker, args=(2, _free_port(), str(tmp_path), refuse),
                           nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        a = torch.load(tmp_path / f"plain{r}.pt", weights_only=True)
        b = torch.load(tmp_path / f"refused{r}.pt", weights_only=True)
        assert b["tried"] == 1 and not b["captured"] and not b["capture_flag"]
        for k in a["state"]:
            assert torch.equal(a["state"][k], b["state"][k]), (r, k)
