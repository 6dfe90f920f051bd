"""hwy_step against hwy_step_group with one handle (development aid): the same env kernel body,
launch parameters from the kernel arguments (by value) or from a device table (by pointer).
Interleaved, 3 rounds, per env count; prints ms per step for each and checks the two produce the
same observations from the same state.

    python tools/probe_step_group1.py [E ...]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "highway-rope-ppo_amd"))
import torch  # noqa: E402

from config.base_config import HIGHWAY_CONFIG  # noqa: E402
from hwy.vec_env import GroupEnvStep, HighwayVecEnv  # noqa: E402

DEV = torch.device("cuda", 0)
for E in [int(x) for x in (sys.argv[1:] or ["4096", "16384"])]:
    envs = [HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device=DEV, autoreset=True, seed_base=42)
            for _ in range(2)]
    for env in envs:
        env.reset()
    bufs = [(torch.zeros(E, 2, device=DEV), torch.empty_like(envs[0].obs_buf),
             torch.empty(E, device=DEV), torch.empty(E, dtype=torch.uint8, device=DEV),
             torch.empty(E, dtype=torch.uint8, device=DEV), None, None) for _ in range(2)]
    g = GroupEnvStep([envs[1]])
    for _ in range(5):
        envs[0].step_into(*bufs[0])
        g.launch([bufs[1]])
    torch.cuda.synchronize()
    same = torch.equal(bufs[0][1], bufs[1][1])
    n = 50
    res = {"hwy_step": [], "hwy_step_group(1)": []}
    for _ in range(3):
        for name in res:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(n):
                if name == "hwy_step":
                    envs[0].step_into(*bufs[0])
                else:
                    g.launch([bufs[1]])
            e.record()
            torch.cuda.synchronize()
            res[name].append(s.elapsed_time(e) / n)
    print(f"E={E} same obs {same}: " + "  ".join(
        f"{k} {min(v):.4f}-{max(v):.4f} ms" for k, v in res.items()), flush=True)
    for env in envs:
        env.close()
