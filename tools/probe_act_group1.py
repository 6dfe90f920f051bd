"""hwy_ppo_act (ActArgs by value) against hwy_ppo_group_act with one learner (arguments from a
device table) -- development aid: microseconds per acting launch at a rollout's row count, and
whether both write the same actions.

    python tools/probe_act_group1.py [rows] [S] [H]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "highway-rope-ppo_amd"))
import torch  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    from hwy.ppo_native import GroupAct, fused_act
    from ppo.agent import PPOAgent

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    torch.manual_seed(0)
    ag = PPOAgent(S, 2, device=DEV, hidden_dim=H)
    st = torch.randn(B, S, device=DEV)
    noise = torch.randn(B, 2, device=DEV)
    o1 = [torch.empty(B, 2, device=DEV), torch.empty(B, 2, device=DEV), torch.empty(B, device=DEV),
          torch.empty(B, device=DEV)]
    o2 = [torch.empty_like(t) for t in o1]
    g = GroupAct([ag], B)
    tiles = g.tiles()
    rows = [(st.data_ptr(), noise.data_ptr()) + tuple(t.data_ptr() for t in o2)]

    def solo():
        fused_act(ag, st, False, None, out=o1, noise=noise)

    def grouped():
        g.launch(rows, tiles)

    solo()
    grouped()
    torch.cuda.synchronize()
    same = all(torch.equal(a, b) for a, b in zip(o1, o2))
    res = {"solo": [], "grouped(1)": []}
    for _ in range(3):
        for name, fn in (("solo", solo), ("grouped(1)", grouped)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 50 * 1e3)
    print(f"rows {B} S {S} H {H} same {same}: " + "  ".join(
        f"{k} {min(v):.2f}-{max(v):.2f} us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
