"""utils.graphs.capture: a garbage collection that would run inside a capture must not destroy a
dead object's graph there.  The child process leaves a reference cycle that owns a captured
graph unreachable, makes every allocation trigger a collection (gc.set_threshold(1)) and then
captures again while allocating Python objects -- the situation that aborted the round-6 GroupBatch
test when an old solo agent's FusedPPO was collected mid-capture.  Run in a child process so a
regression aborts the child, not the test session."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import gc, sys
sys.path.insert(0, sys.argv[1])
import torch
from utils.graphs import capture

class Owner:
    pass

def captured(x):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with capture(g, stream=s, collect=False):
            junk = [Owner() for _ in range(2000)]  # allocations: collections if gc were on
            x.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    return g

x = torch.zeros(4, device="cuda")
o = Owner()
o.me, o.graph = o, captured(x)  # a cycle owning a graph
del o                           # unreachable, not yet collected
gc.set_threshold(1)
g = captured(x)
g.replay()
torch.cuda.synchronize()
assert gc.isenabled()
print("ok", float(x.sum()))
"""


@pytest.mark.gpu
def test_capture_holds_collector_off_while_capturing():
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "highway-rope-ppo_amd")],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip() == "ok 4.0", r.stdout


def test_capture_restores_the_collector_when_capture_fails():
    """No GPU here: torch refuses the capture, and the collector comes back on."""
    import gc

    sys.path.insert(0, os.path.join(ROOT, "highway-rope-ppo_amd"))
    from utils.graphs import capture

    assert gc.isenabled()
    with pytest.raises(Exception):
        with capture(None):
            pass
    assert gc.isenabled()
