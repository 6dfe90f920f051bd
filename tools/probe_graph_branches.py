"""Do the independent branches of one HIP graph run concurrently on gfx950 / ROCm 7?

G chains of K small dependent kernels each (one 256-thread workgroup per launch, ~a few us of
work), issued four ways, timed with HIP events:
  serial   one stream, the G chains one after another, captured as one graph
  branches one graph captured fork-join: chain g on its own forked stream (G parallel branches)
  streams  G streams, each replaying its own one-chain graph (HW queues: GPU_MAX_HW_QUEUES)
  eager    the serial order, eager launches
Prints microseconds per replay and the speed-up over serial."""
import sys

import torch

G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
dev = torch.device("cuda", 0)
xs = [torch.zeros(256 * 64, device=dev) for _ in range(G)]


def chain(x):
    for _ in range(K):
        x.mul_(1.0001).add_(1.0)  # two small dependent launches per link


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


# serial graph
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g_serial = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    for x in xs:
        chain(x)  # warm
    torch.cuda.synchronize()
    with torch.cuda.graph(g_serial, stream=s):
        for x in xs:
            chain(x)
torch.cuda.current_stream().wait_stream(s)
t_serial = timed(g_serial.replay)

# fork-join graph: each chain on its own stream inside the capture
g_br = torch.cuda.CUDAGraph()
side = [torch.cuda.Stream() for _ in range(G)]
with torch.cuda.graph(g_br, stream=s):
    root = torch.cuda.current_stream()
    for st, x in zip(side, xs):
        st.wait_stream(root)
        with torch.cuda.stream(st):
            chain(x)
    for st in side:
        root.wait_stream(st)
t_br = timed(g_br.replay)

# G streams, each its own graph
graphs = []
for st, x in zip(side, xs):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            chain(x)
    graphs.append((st, g))


def multi():
    cur = torch.cuda.current_stream()
    for st, g in graphs:
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            g.replay()
    for st, _ in graphs:
        cur.wait_stream(st)


t_streams = timed(multi)
t_eager = timed(lambda: [chain(x) for x in xs], reps=3)
print(f"G={G} K={K} launches/replay={2 * G * K}")
for name, t in (("serial", t_serial), ("branches", t_br), ("streams", t_streams), ("eager", t_eager)):
    print(f"{name:9s} {t:10.1f} us  x{t_serial / t:5.2f}  ({t / (2 * G * K):.2f} us/launch)")
