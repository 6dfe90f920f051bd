"""Drift of the product update (PPOAgent.update_rollout -> hwy_gae -> FusedPPO) against the
reference's golden updates at the benched learners (tests/golden/ppo_agent_bench.npz): per
parameter the max |diff| and the share of elements past a few thresholds, and every metric's
difference.  Sets the tolerances of test_fused_update_replays_reference_golden_bench."""
import json
import sys

import numpy as np
import torch

sys.path[:0] = ["tests", "highway-rope-ppo_amd", "."]
from agent_util import load  # noqa: E402
from ppo.agent import PPOAgent, RolloutBuffer  # noqa: E402

DEV = torch.device("cuda", 0)
g, meta = load(bench=True)
res = {}
for name in sys.argv[1:] or ["upd_c1", "upd_c2", "upd_c4"]:
    for backend, graphs in (("hip", False), ("hip", True), ("torch", False)):
        m = meta["agent"][name]
        n, S = m["n"], m["state_dim"]
        agent = PPOAgent(S, 2, lr=m["lr"], epochs=m["epochs"], batch_size=m["batch_size"],
                         hidden_dim=m["hidden_dim"], device=DEV, use_graphs=graphs, backend=backend)
        sd = {k[len(name) + 6:]: torch.as_tensor(g[k]) for k in g.files if k.startswith(f"{name}_init_")}
        agent.actor_critic.load_state_dict(sd)
        buf = RolloutBuffer(n, 1, S, 2, DEV)
        f = lambda k: torch.as_tensor(np.asarray(g[f"{name}_{k}"], np.float32), device=DEV)  # noqa: E731
        buf.states[:n].copy_(f("states").view(n, 1, S))
        buf.actions.copy_(f("actions").view(n, 1, 2))
        buf.pre_tanh.copy_(f("pre_tanh").view(n, 1, 2))
        buf.log_probs.copy_(f("log_probs").view(n, 1))
        buf.values.copy_(f("values").view(n, 1))
        buf.rewards.copy_(f("rewards").view(n, 1))
        buf.dones.copy_(torch.as_tensor(np.asarray(g[f"{name}_dones"], np.uint8), device=DEV).view(n, 1))
        perm = torch.as_tensor(np.asarray(g[f"{name}_perm"], np.int64), device=DEV)
        last = torch.tensor([m["last_value"]], dtype=torch.float32, device=DEV)
        metrics = agent.update_rollout(buf, last, perm=perm)
        F = getattr(agent, "_fused", None)
        out = {"fused": F is not None, "mb": F.mb if F else None, "nmb": F.nmb if F else None}
        for k, v in agent.actor_critic.state_dict().items():
            want = g[f"{name}_final_{k}"]
            d = np.abs(v.detach().cpu().numpy() - want)
            scale = np.abs(want).max()
            out[k] = {"max": float(d.max()), "p999": float(np.quantile(d, 0.999)),
                      "gt1e-5": float((d > 1e-5).mean()), "gt1e-4": float((d > 1e-4).mean()),
                      "rel_norm": float(np.linalg.norm(d) / max(np.linalg.norm(want), 1e-30)),
                      "scale": float(scale)}
        out["metrics"] = {k: [metrics[k], want, abs(metrics[k] - want)] for k, want in m["metrics"].items()}
        res[f"{name}_{backend}_graphs{int(graphs)}"] = out
        print(name, backend, graphs, json.dumps(out["metrics"]), flush=True)
        for k, v in out.items():
            if isinstance(v, dict) and "max" in v:
                print(f"   {k:22s} max {v['max']:.2e} p999 {v['p999']:.2e} >1e-5 {v['gt1e-5']:.4f} "
                      f">1e-4 {v['gt1e-4']:.4f} relnorm {v['rel_norm']:.2e}", flush=True)
json.dump(res, open("gpurun_out/golden_bench_drift.json", "w"), indent=1)
