"""Per-minibatch-step time of the fused update on the distributed path (graph -> RCCL
all-reduce -> graph) with a 1-rank RCCL group, against the single-graph path (development
aid: shows the host-side cost the N > 1 structure adds on one GPU)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
from hwy.ppo_native import FusedPPO
from ppo.agent import PPOAgent

S, H, mb, nmb = 60, 256, 4096, 32
n = mb * nmb
torch.manual_seed(0)
s = torch.randn(n, S, device=dev)
z = torch.randn(n, 2, device=dev)
lp = torch.randn(n, device=dev) - 2
adv = torch.randn(n, device=dev)
ret = torch.randn(n, device=dev)
perm = torch.randperm(n, device=dev)
for group in (None, dist.group.WORLD):
    ag = PPOAgent(S, 2, lr=3e-4, epochs=2, hidden_dim=H, device=dev, backend="hip")
    F = FusedPPO(ag, mb, nmb, group=group, use_graphs=True)
    F.run(s, z, lp, adv, ret, perm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(3):
        F.run(s, z, lp, adv, ret, perm)
    e1.record()
    host = (time.perf_counter() - t0) / (3 * 2 * nmb) * 1e6
    torch.cuda.synchronize()
    gpu = e0.elapsed_time(e1) / (3 * 2 * nmb) * 1e3
    print(f"{'single graph' if group is None else 'rccl 1-rank '}: {gpu:.1f} us per step (GPU), "
          f"host issue {host:.1f} us per step", flush=True)
dist.destroy_process_group()
