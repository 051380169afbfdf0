"""HIP-graph capture of whole training steps (no tracing compiler, just replay).

A train step of the layer-by-layer models (LSTM stack, MLP) is ~40 kernel launches:
the fused layer kernels plus small ones (loss, slab reductions, autograd gradient
accumulation, Adam). Run eagerly, every launch pays the host dispatch and the
inter-kernel gap. Captured once into a HIP graph (``torch.cuda.CUDAGraph`` is the
ROCm hipGraph), each step is ONE replay.

The step callables must be capture-safe:
* no host synchronisation (``.item()``, ``.cpu()``);
* inputs at fixed addresses (each callable closes over its own batch view);
* parameters and gradients updated in place. ``FlatParams`` / ``FlatAdam`` already do
  this: the gradients are views of one flat buffer that autograd accumulates into, and
  Adam updates the flat buffer with the step counter on the device.

Returns a function ``step(s)`` that replays graph ``s % len(fns)`` and returns that
graph's (static) outputs.
"""
from __future__ import annotations

from typing import Callable, List, Sequence

import torch


def capture_steps(fns: Sequence[Callable[[], object]], warmup: int = 2) -> Callable[[int], object]:
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):   # allocator / autograd warm-up off the capture stream
        for _ in range(warmup):
            for f in fns:
                f()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graphs: List[torch.cuda.CUDAGraph] = []
    outs: List[object] = []
    pool = None
    for f in fns:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            outs.append(f())
        pool = g.pool()   # the graphs share one memory pool (they never run concurrently)
        graphs.append(g)
    torch.cuda.synchronize()

    def step(s: int):
        k = s % len(graphs)
        graphs[k].replay()
        return outs[k]

    return step
