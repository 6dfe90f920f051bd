"""Fused and torch-fp32 gradients against a float64 autograd reference (diagnostic)."""
import sys, os, copy
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "highway-rope-ppo_amd"), os.path.join(ROOT, "tests")]
import torch
import torch.nn.functional as Fn
from torch.distributions import Normal
from test_ppo_fused_gpu import _agents, _data, _torch_grad
from hwy.ppo_native import FusedPPO


def grad64(ac, s, z, lp, adv, ret, idx, eps=0.2, vc=0.5, ec=0.005):
    m = copy.deepcopy(ac).double()
    s, z, lp, adv, ret = (t.double()[idx] for t in (s, z, lp, adv, ret))
    mean, std, v = m(s)
    dist = Normal(mean, std, validate_args=False)
    a = torch.tanh(z)
    nlp = (dist.log_prob(z) - torch.log1p(-a.pow(2) + 1e-6)).sum(-1)
    r = torch.exp(nlp - lp)
    loss = (-torch.min(r * adv, torch.clamp(r, 1 - eps, 1 + eps) * adv).mean()
            + vc * Fn.mse_loss(v.squeeze(-1), ret) - ec * dist.entropy().sum(-1).mean())
    loss.backward()
    return {n: p.grad for n, p in m.named_parameters()}


for S, H, mb in [(240, 512, 4096), (240, 256, 4096), (60, 256, 4096)]:
    a, b = _agents(S, H)
    s, z, lp, adv, ret, perm = _data(mb * 2, S, a)
    idx = perm[:mb].contiguous()
    g64 = grad64(a.actor_critic, s, z, lp, adv, ret, idx)
    _torch_grad(a, s, z, lp, adv, ret, idx)
    F = FusedPPO(b, mb, 2, use_graphs=False)
    args = F._args(s, z, lp, adv, ret, idx.data_ptr())
    F.counters.zero_(); F.sync_params(args); F._fwd_bwd(args); torch.cuda.synchronize()
    ga, gb = dict(a.actor_critic.named_parameters()), dict(b.actor_critic.named_parameters())
    for n in ga:
        r = g64[n]
        et = (ga[n].grad.double() - r).abs()
        ef = (gb[n].grad.double() - r).abs()
        i = int(ef.argmax())
        rows = torch.nonzero(ef > 10 * et.max()).tolist()[:8]
        print(S, H, n, "torch_err %.3e fused_err %.3e | at %d ref64 %.5e torch %.5e fused %.5e | n_fused>10x_torchmax %d %s" % (
            et.max(), ef.max(), i, r.reshape(-1)[i], ga[n].grad.reshape(-1)[i], gb[n].grad.reshape(-1)[i],
            int((ef > 10 * et.max()).sum()), rows), flush=True)
