"""Diagnose the 1-rank RCCL epoch-graph capture's teardown (tests/test_dist_fused_gpu.py::
test_rccl_captured_allreduce_matches_stepwise_and_local aborted in ~CUDAGraph with "operation not
permitted when stream is capturing").  argv[1]:
  locals   the worker's body inside a function, destroy_process_group before the locals die
  release  the same, but every FusedPPO's graphs released (FusedPPO.release_graphs) first"""
import gc
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(here), "highway-rope-ppo_amd"),
                os.path.join(os.path.dirname(here), "tests")]
mode = sys.argv[1] if len(sys.argv) > 1 else "locals"
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("PORT", "29611"))


def body():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from hwy.ppo_native import FusedPPO
    from test_dist_fused_gpu import NLOC, NMB, _agent, _data

    d = _data(0, dev)
    keep = []
    for tag, group, capture in (("captured", torch.distributed.group.WORLD, True),
                                ("stepwise", torch.distributed.group.WORLD, False),
                                ("local", None, False)):
        agent = _agent(dev, group)
        adv = agent.normalize_advantages(d["a"])
        F = FusedPPO(agent, NLOC // NMB, NMB, group=group, use_graphs=True)
        F.capture_collectives = capture
        for _ in range(2):
            F.run(d["s"], d["z"].contiguous(), d["lp"], adv.contiguous(), d["r"], d["perm"])
        torch.cuda.synchronize()
        print(tag, "captured", F._captured_collectives, flush=True)
        keep.append(F)
    if mode == "release":
        for F in keep:
            F.release_graphs()
    print("destroying the process group", flush=True)
    torch.distributed.destroy_process_group()
    print("destroyed; returning", flush=True)


body()
gc.collect()
print("exit ok", flush=True)
