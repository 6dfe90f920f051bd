"""Development probe: does a rollout graph with two env halves on two streams (act of one half
overlapping the env step of the other) beat the single-stream rollout graph?

  python tools/r2/split_probe.py [E] [T] [reps]
"""

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "highway-rope-ppo_amd"))

import torch  # noqa: E402

from hwy import native  # noqa: E402

if os.environ.get("HWY_LIB"):  # a variant library (development A/B)
    native.LIB_PATH = os.environ["HWY_LIB"]
from config.base_config import HIGHWAY_CONFIG  # noqa: E402
from experiments.config import Condition  # noqa: E402
from experiments.wrappers import make_env  # noqa: E402
from ppo.agent import PPOAgent, RolloutBuffer  # noqa: E402
from ppo.rollout import LockstepRollout  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
T = int(sys.argv[2]) if len(sys.argv) > 2 else 128
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda", 0)
torch.manual_seed(1234)


def mk(n, off):
    w = make_env(Condition.SORTED, HIGHWAY_CONFIG,
                 env_overrides={"observation": {"vehicles_count": 15, "order": "sorted"},
                                "num_envs": n, "device": dev, "autoreset": True,
                                "env_offset": off, "global_envs": E})
    env = w.unwrapped
    env.set_seed_schedule(42)
    return env


env = mk(E, 0)
sd = env.obs_rows * env.obs_features
agent = PPOAgent(sd, 2, lr=3e-4, epochs=8, batch_size=64, hidden_dim=256, device=dev,
                 num_minibatches=32, seed=1000)
buf = RolloutBuffer(T, E, sd, 2, dev)
buf.states[0].copy_(env.reset()[0].reshape(E, sd))
roll = LockstepRollout(agent, env, buf)

halves = []
for h in range(2):
    e = mk(E // 2, h * E // 2)
    b = RolloutBuffer(T, E // 2, sd, 2, dev)
    b.states[0].copy_(e.reset()[0].reshape(E // 2, sd))
    halves.append((e, b, LockstepRollout(agent, e, b, use_graph=False)))


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / REPS * 1e3


print(f"single stream graph, E={E}: {timeit(roll.run):.3f} ms per rollout of {T}")
if os.environ.get("SPLIT", "1") == "0":
    sys.exit(0)

# two halves, each its own chain, captured into one graph on two streams
for _, b, _ in halves:
    b.draw_noise(agent.generator)
for _, _, r in halves:  # eager warm-up (allocations)
    r._steps()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
s1.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s1):
    with torch.cuda.graph(g, stream=s1):
        s2.wait_stream(s1)
        with torch.cuda.stream(s2):
            halves[1][2]._steps()
        halves[0][2]._steps()
        s1.wait_stream(s2)
torch.cuda.current_stream().wait_stream(s1)
print(f"two-stream graph, 2 x {E // 2}: {timeit(g.replay):.3f} ms per rollout of {T}")

g2 = torch.cuda.CUDAGraph()
with torch.cuda.stream(s1):
    with torch.cuda.graph(g2, stream=s1):
        halves[0][2]._steps()
        halves[1][2]._steps()
torch.cuda.current_stream().wait_stream(s1)
print(f"one-stream graph, 2 x {E // 2} in sequence: {timeit(g2.replay):.3f} ms")
