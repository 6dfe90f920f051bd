"""Times the fused PPO update (graph of ppo_rows / ppo_wgrad / ppo_wsum / ppo_adam) at the bench
minibatch (development aid): probe_ppo_time.py [H] [reps] [minibatch rows] [S]; HWY_LIB
overrides the library; PROBE_KT=1 also prints each kernel's time (hwy_ppo_time_kernels)."""
import os, sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import torch
import hwy.native as native

if os.environ.get("HWY_LIB"):
    native.LIB_PATH = os.environ["HWY_LIB"]
from hwy.ppo_native import FusedPPO
from ppo.agent import PPOAgent

dev = torch.device("cuda", 0)
S = int(sys.argv[4]) if len(sys.argv) > 4 else 60
H, nmb = int(sys.argv[1]) if len(sys.argv) > 1 else 256, 32
mb = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
torch.manual_seed(0)
ag = PPOAgent(S, 2, lr=3e-4, epochs=1, hidden_dim=H, device=dev, use_graphs=False, backend="hip")
n = mb * nmb
s = torch.randn(n, S, device=dev)
z = torch.randn(n, 2, device=dev)
lp = torch.randn(n, device=dev) - 2
adv = torch.randn(n, device=dev)
ret = torch.randn(n, device=dev)
perm = torch.randperm(n, device=dev)
F = FusedPPO(ag, mb, nmb, use_graphs=True)
F.run(s, z, lp, adv, ret, perm)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(reps):
    F.run(s, z, lp, adv, ret, perm)
ev1.record()
torch.cuda.synchronize()
print(f"H={H}: {ev0.elapsed_time(ev1) / (reps * nmb) * 1e3:.1f} us per minibatch step", flush=True)
if os.environ.get("PROBE_KT"):  # per-kernel times (hwy_ppo_time_kernels), after the timed loop
    kt = F.time_kernels(16)
    print("per kernel us: " + " ".join(f"{k} {v:.2f}" for k, v in kt.items()), flush=True)
# bit-identity fingerprint of the final weights (variants that only reorder instructions must
# print the same value as the product library)
import hashlib

print(f"weights sha1 {hashlib.sha1(F.flat.detach().cpu().numpy().tobytes()).hexdigest()[:16]}", flush=True)
