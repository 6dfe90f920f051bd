"""Rollout timing: one E-env handle on one stream vs K handles of E/K envs on K streams
(each half's act overlapping the other half's env step).  Development aid."""
import os, sys, time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import torch
from config.base_config import HIGHWAY_CONFIG
from hwy.vec_env import HighwayVecEnv
from ppo.agent import PPOAgent, RolloutBuffer

dev = torch.device("cuda", 0)
E, T = 4096, 32
K = int(sys.argv[1]) if len(sys.argv) > 1 else 2
agent = PPOAgent(60, 2, hidden_dim=256, device=dev, seed=0)
buf = RolloutBuffer(T, E, 60, 2, dev)


def run(envs, streams, reps=5):
    n = E // len(envs)
    obs0 = []
    for k, env in enumerate(envs):
        o, _ = env.reset()
        buf.states[0][k * n:(k + 1) * n].copy_(o.reshape(n, 60))
    torch.cuda.synchronize()
    times = []
    for r in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        buf.draw_noise(agent.generator)
        main = torch.cuda.current_stream()
        for s in streams:
            s.wait_stream(main)
        for t in range(T):
            for k, (env, s) in enumerate(zip(envs, streams)):
                sl = slice(k * n, (k + 1) * n)
                with torch.cuda.stream(s):
                    agent.select_action(buf.states[t][sl], out=(buf.actions[t][sl], buf.pre_tanh[t][sl],
                                                                buf.log_probs[t][sl], buf.values[t][sl]),
                                        noise=buf.noise[t][sl])
                    env.step_into(buf.actions[t][sl], buf.states[t + 1][sl], buf.rewards[t][sl],
                                  buf.terminated[t][sl], buf.truncated[t][sl], buf.ep_return[t][sl],
                                  buf.ep_length[t][sl])
        for s in streams:
            main.wait_stream(s)
        torch.cuda.synchronize()
        if r:
            times.append(time.perf_counter() - t0)
        buf.states[0].copy_(buf.states[T])
    return 1e3 * sum(times) / len(times)


one = [HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device=dev, seed_base=42)]
ms1 = run(one, [torch.cuda.current_stream()])
one[0].close()
envs = [HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E // K, device=dev, seed_base=42,
                      env_offset=k * (E // K), global_envs=E) for k in range(K)]
msK = run(envs, [torch.cuda.Stream() for _ in range(K)])
msK1 = run(envs, [torch.cuda.current_stream()] * K)
print(f"rollout T={T} E={E}: 1 handle {ms1:.2f} ms; {K} handles on {K} streams {msK:.2f} ms; "
      f"{K} handles on 1 stream {msK1:.2f} ms")
