"""Times hwy_ppo_act from the update's tile image (development aid): probe_act.py [rows ...];
HWY_LIB overrides the library."""
import os, sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import torch
import hwy.native as native

if os.environ.get("HWY_LIB"):
    native.LIB_PATH = os.environ["HWY_LIB"]
from hwy.ppo_native import FusedPPO, fused_act
from ppo.agent import PPOAgent

dev = torch.device("cuda", 0)
S, H = (int(v) for v in os.environ.get("HWY_PROBE_SH", "60:256").split(":"))
n = 16384
torch.manual_seed(0)
ag = PPOAgent(S, 2, lr=3e-4, epochs=1, hidden_dim=H, device=dev, use_graphs=False, backend="hip")
s = torch.randn(n, S, device=dev); z = torch.randn(n, 2, device=dev)
lp = torch.randn(n, device=dev) - 2; adv = torch.randn(n, device=dev); ret = torch.randn(n, device=dev)
F = FusedPPO(ag, n, 1, use_graphs=False)
ag._fused = F
F.run(s, z, lp, adv, ret, torch.randperm(n, device=dev))
assert F.current_tiles(F.flat) is not None
for B in [int(x) for x in (sys.argv[1:] or ["4096", "16384"])]:
    x = torch.randn(B, S, device=dev)
    noise = torch.randn(B, 2, device=dev)
    out = (torch.empty(B, 2, device=dev), torch.empty(B, 2, device=dev), torch.empty(B, device=dev),
           torch.empty(B, device=dev))
    for _ in range(20):
        fused_act(ag, x, noise=noise, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 200
    e0.record()
    for _ in range(reps):
        fused_act(ag, x, noise=noise, out=out)
    e1.record()
    torch.cuda.synchronize()
    print(f"B={B}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us per act (incl. launch)", flush=True)
