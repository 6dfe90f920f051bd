"""Development probe: the fused step's intermediate row outputs (h1, h2, dac, dh2, dh1 in the
workspace) against float64 autograd on the same minibatch, per 128-column block.

  python tools/r2/probe_dac.py S H rows
"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "highway-rope-ppo_amd"))
import torch  # noqa: E402
import torch.nn.functional as Fn  # noqa: E402
from torch.distributions import Normal  # noqa: E402

import test_ppo_fused_gpu as T  # noqa: E402

S, H, mb = (int(x) for x in sys.argv[1:4])
a, b = T._agents(S, H)
s, z, lp, adv, ret, perm = T._data(2 * mb, S, a)
idx = perm[:mb].contiguous()
F = T.FusedPPO(b, mb, 2, use_graphs=False)
args = F._args(s, z, lp, adv, ret, idx.data_ptr())
F.counters.zero_()
F.sync_params(args)
F._fwd_bwd(args)
torch.cuda.synchronize()

# float64 reference with the intermediate gradients
m = copy.deepcopy(a.actor_critic).double()
acts = {}


def keep(name):
    def hook(mod, inp, out):
        out.retain_grad()
        acts[name] = out
    return hook


m.shared[1].register_forward_hook(keep("h1"))
m.shared[3].register_forward_hook(keep("h2"))
m.shared[0].register_forward_hook(keep("z1"))
m.shared[2].register_forward_hook(keep("z2"))
m.actor_mean[0].register_forward_hook(keep("za"))
m.critic[0].register_forward_hook(keep("zc"))
sd, zd, lpd, advd, retd = (t.double()[idx] for t in (s, z, lp, adv, ret))
mean, std, v = m(sd)
dist = Normal(mean, std, validate_args=False)
nlp = (dist.log_prob(zd) - torch.log1p(-torch.tanh(zd).pow(2) + 1e-6)).sum(-1)
r = torch.exp(nlp - lpd)
loss = (-torch.min(r * advd, torch.clamp(r, 1 - a.eps_clip, 1 + a.eps_clip) * advd).mean()
        + a.value_coef * Fn.mse_loss(v.squeeze(-1), retd)
        - a.entropy_coef * dist.entropy().sum(-1).mean())
loss.backward()
ref = {"h1": acts["h1"].detach(), "h2": acts["h2"].detach(),
       "dac": torch.cat([acts["za"].grad, acts["zc"].grad], 1),
       "dh2": acts["z2"].grad, "dh1": acts["z1"].grad}

ws = F.workspace.view(torch.float32)
sizes = [("h1", mb * H), ("h2", mb * H), ("ac", mb * 2 * H), ("dac", mb * 2 * H),
         ("dh2", mb * H), ("dh1", mb * H)]
off = 0
for name, n in sizes:
    width = n // mb
    got = ws[off:off + n].view(mb, width).double()
    off += (n + 63) // 64 * 64
    if name not in ref:
        continue
    e = (got - ref[name]).abs()
    sc = ref[name].abs().max().item()
    blocks = [e[:, c:c + 128].max().item() / sc for c in range(0, width, 128)]
    i, j = divmod(int(e.argmax()), width)
    print(f"{name:4s} max|ref| {sc:.3e}  rel err per 128-col block "
          + " ".join(f"{x:.1e}" for x in blocks) + f"  worst at row {i} col {j}")
    bad = (e > 1e-4 * sc).nonzero()
    if len(bad):
        rows = bad[:, 0].unique()
        print(f"     {len(bad)} elements > 1e-4 rel in {len(rows)} rows; rows mod 16: "
              f"{sorted(set((rows % 16).tolist()))[:16]}, first rows {rows[:8].tolist()}, "
              f"cols {sorted(set(bad[:, 1].tolist()))[:8]}..")
