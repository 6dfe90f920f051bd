"""Development probe: per-parameter errors of the fused gradient at (S, H, rows) against float64
autograd and torch fp32 (tests/test_ppo_fused_gpu.py's check, printed instead of asserted)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "highway-rope-ppo_amd"))
import torch  # noqa: E402
import test_ppo_fused_gpu as T  # noqa: E402

S, H, mb = (int(x) for x in sys.argv[1:4])
a, b = T._agents(S, H)
s, z, lp, adv, ret, perm = T._data(2 * mb, S, a)
idx = perm[:mb].contiguous()
g64 = T._grad64(a, s, z, lp, adv, ret, idx)
T._torch_grad(a, s, z, lp, adv, ret, idx)
F = T.FusedPPO(b, mb, 2, use_graphs=False)
args = F._args(s, z, lp, adv, ret, idx.data_ptr())
F.counters.zero_()
F.sync_params(args)
F._fwd_bwd(args)
torch.cuda.synchronize()
ga = dict(a.actor_critic.named_parameters())
gb = dict(b.actor_critic.named_parameters())
for name, pa in ga.items():
    ref = g64[name]
    t32 = pa.grad.double()
    got = gb[name].grad.double()
    scale = max(ref.abs().max().item(), 1e-3)
    ok64 = torch.allclose(got, ref, rtol=1e-3, atol=2e-5 * scale)
    ok32 = torch.allclose(got, t32, rtol=1e-3, atol=2e-5 * scale)
    ef = (got - ref).abs().max().item()
    et = (t32 - ref).abs().max().item()
    print(f"{name:24s} scale {scale:.3e} e_fused {ef:.3e} e_torch {et:.3e} ok64 {ok64} ok32 {ok32} "
          f"bound2 {ef <= 2 * et + 2e-5 * scale}")

for name in ("critic.0.weight", "shared.0.weight"):
    ref = g64[name]
    got = gb[name].grad.double()
    err = (got - ref).abs()
    i, j = divmod(int(err.argmax()), err.shape[1])
    print(f"{name}: max|ref| {ref.abs().max().item():.3e}, max err at ({i}, {j}) = {err.max().item():.3e},"
          f" ref there {ref[i, j].item():.3e} got {got[i, j].item():.3e}")
    rb = err.shape[0] // 128 if err.shape[0] >= 128 else 1
    blk = err[: rb * 128].reshape(rb, -1, err.shape[1]).amax(dim=(1, 2)) if rb > 1 else err.amax()
    print("  max err per 128-row block:", [f"{v:.1e}" for v in (blk.tolist() if rb > 1 else [blk.item()])])
