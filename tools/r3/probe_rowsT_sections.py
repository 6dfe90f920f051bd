"""Per-phase shader clocks of ppo_rowsT (development aid; profiling build, make prof):
probe_rowsT_sections.py [H] [minibatch rows] [S]"""
import ctypes, os, sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "highway-rope-ppo_amd"))
import torch
import hwy.native as native

native.LIB_PATH = os.path.join(os.path.dirname(native.LIB_PATH), "libhwy_prof.so")
from hwy.ppo_native import FusedPPO
from ppo.agent import PPOAgent

dev = torch.device("cuda", 0)
H = int(sys.argv[1]) if len(sys.argv) > 1 else 256
mb = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
S = int(sys.argv[3]) if len(sys.argv) > 3 else 60
nmb = 8
torch.manual_seed(0)
ag = PPOAgent(S, 2, lr=3e-4, epochs=1, hidden_dim=H, device=dev, use_graphs=False, backend="hip")
n = mb * nmb
s = torch.randn(n, S, device=dev); z = torch.randn(n, 2, device=dev)
lp = torch.randn(n, device=dev) - 2; adv = torch.randn(n, device=dev); ret = torch.randn(n, device=dev)
perm = torch.randperm(n, device=dev)
F = FusedPPO(ag, mb, nmb, use_graphs=True)
L = native.lib()
L.hwy_ppo_debug_sections.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
F.run(s, z, lp, adv, ret, perm); torch.cuda.synchronize()
L.hwy_ppo_debug_sections(buf, 1)
reps = 4
F.run(s, z, lp, adv, ret, perm)
for _ in range(reps - 1):
    F.run(s, z, lp, adv, ret, perm)
torch.cuda.synchronize()
L.hwy_ppo_debug_sections(buf, 1)
n1 = mb // 64
steps = reps * nmb
names = {0: "prologue", 1: "h1 stages", 2: "h2 stages", 3: "a/c stages", 13: "epilogues",
         7: "loss head", 4: "head sync", 5: "dh2 stages", 6: "dh1 stages", 12: "stage barriers"}
tot = sum(buf[i] for i in names)
for i, nm in names.items():
    print(f"  {nm:16s} {buf[i] / (steps * n1):10,.0f} clk/WG  {100 * buf[i] / tot:5.1f}%")
NG = H // 16
sb = ((S + 15) // 16 + 3) // 4 * 4
floor = (sb * NG + 6 * NG * NG) * 4 * 32  # v_mfma_f32_16x16x4_f32 per wave x 32 cycles
print(f"  total {tot / (steps * n1):,.0f} clk/WG (wave 0); MFMA issue floor {floor:,} clk")
