"""FusedPPO's minibatch step as its solo kernels (arguments by value) against the grouped kernels
with one learner (arguments read from a device table, hwy_ppo_group_step) -- development aid.
One epoch of 32 minibatch steps captured as a graph each way, replayed interleaved; prints the
microseconds per minibatch step and whether both leave the same weights.

    python tools/probe_ppo_group1.py [rows] [S] [H]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "highway-rope-ppo_amd"))
import torch  # noqa: E402

from utils.graphs import capture  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    from hwy.ppo_native import FusedPPO, GroupStep
    from ppo.agent import PPOAgent

    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    nmb = 32
    n = mb * nmb
    torch.manual_seed(0)
    agent = PPOAgent(S, 2, lr=3e-4, epochs=1, batch_size=64, hidden_dim=H, device=DEV,
                     num_minibatches=nmb, backend="hip")
    g = torch.Generator(device=DEV).manual_seed(1)
    st = torch.randn(n, S, device=DEV, generator=g)
    z = torch.randn(n, 2, device=DEV, generator=g) * 0.5
    lp = torch.randn(n, device=DEV, generator=g) - 2.0
    adv = torch.randn(n, device=DEV, generator=g)
    ret = torch.randn(n, device=DEV, generator=g)
    perm = torch.randperm(n, device=DEV, generator=g)
    F = FusedPPO(agent, mb, nmb, use_graphs=False)
    F.run(st, z, lp, adv, ret, perm)
    torch.cuda.synchronize()
    args = F._last_args
    step = GroupStep([F])
    step.prepare([args])
    snap = [t.clone() for t in (F.flat, F.m, F.v, F.counters)]

    def restore():
        for t, s in zip((F.flat, F.m, F.v, F.counters), snap):
            t.copy_(s)
        F.sync_params(args[0])

    graphs = {}
    for name in ("solo (kernel arguments)", "grouped, G = 1 (device table)"):
        gr = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with capture(gr, stream=s):
                for i, a in enumerate(args):
                    if name.startswith("solo"):
                        F._fwd_bwd(a)
                        F._opt(a)
                    else:
                        step.step(i)
        torch.cuda.current_stream().wait_stream(s)
        graphs[name] = gr
    out = {}
    for name, gr in graphs.items():
        restore()
        F.counters[1].zero_()
        gr.replay()
        torch.cuda.synchronize()
        out[name] = F.flat.clone()
    same = torch.equal(*out.values())
    res = {k: [] for k in graphs}
    for _ in range(5):
        for name, gr in graphs.items():
            restore()
            F.counters[1].zero_()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / nmb * 1e3)
    print(f"rows {mb} S {S} H {H}: same weights {same}", flush=True)
    for k, v in res.items():
        print(f"  {k:32s} {min(v):7.2f} - {max(v):7.2f} us per minibatch step", flush=True)


if __name__ == "__main__":
    main()
