"""HIP graph capture with the cyclic garbage collector held off.

A collection that runs while a stream is capturing can free an unrelated, unreachable object
that owns a captured graph (an old agent's FusedPPO, a finished rollout): its destructor then
destroys a graph executable mid-capture, which the runtime refuses ("operation not permitted
when stream is capturing") and torch turns into an abort.  torch.cuda.graph no longer collects
before capturing (torch.compiler.config.force_cudagraph_gc is off by default), so this collects
first -- dead graphs are destroyed while nothing captures -- and holds the collector off for the
capture itself.  Captures happen once per argument key, so the collection's cost is off the
replayed path.
"""

from __future__ import annotations

import contextlib
import gc

import torch


@contextlib.contextmanager
def capture(graph: torch.cuda.CUDAGraph, stream=None, collect: bool = True, **kw):
    """torch.cuda.graph(graph, stream=stream, **kw), after a collection (collect=False: the
    caller has just collected, e.g. before a run of back-to-back captures) and with gc disabled
    inside."""
    if collect:
        gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(graph, stream=stream, **kw):
            yield graph
    finally:
        if was:
            gc.enable()
