"""Fused-vs-autograd gradient error statistics per parameter (diagnostic for
tests/test_ppo_fused_gpu.py::test_fused_gradient_matches_autograd)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "highway-rope-ppo_amd"), os.path.join(ROOT, "tests")]
import torch
from test_ppo_fused_gpu import _agents, _data, _torch_grad
from hwy.ppo_native import FusedPPO

for S, H, mb in [(60, 256, 4096), (120, 384, 4096), (240, 256, 4096), (240, 512, 4096), (240, 256, 256), (136, 128, 128)]:
    a, b = _agents(S, H)
    s, z, lp, adv, ret, perm = _data(mb * 2, S, a)
    idx = perm[:mb].contiguous()
    _torch_grad(a, s, z, lp, adv, ret, idx)
    F = FusedPPO(b, mb, 2, use_graphs=False)
    args = F._args(s, z, lp, adv, ret, idx.data_ptr())
    F.counters.zero_(); F.sync_params(args); F._fwd_bwd(args); torch.cuda.synchronize()
    ga, gb = dict(a.actor_critic.named_parameters()), dict(b.actor_critic.named_parameters())
    for n, p in ga.items():
        r, g = p.grad, gb[n].grad
        d = (g - r).abs()
        scale = max(r.abs().max().item(), 1e-3)
        bad = (d > 1e-3 * r.abs() + 2e-5 * scale)
        i = int(d.argmax())
        print(S, H, mb, n, "scale %.3e maxd %.3e rel %.2e bad %d/%d at %d ref %.4e got %.4e" % (
            scale, d.max().item(), d.max().item() / scale, int(bad.sum()), d.numel(), i,
            r.reshape(-1)[i].item(), g.reshape(-1)[i].item()), flush=True)
