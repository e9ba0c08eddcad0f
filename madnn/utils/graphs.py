"""Whole-step HIP-graph capture: one graph launch per training step instead of ~650 kernel launches.

A ResNet-50 step at a small per-GPU batch is a few hundred short kernels; the host enqueues them
one by one and the GPU idles whenever the host falls behind.  :func:`capture_step` records the
ENTIRE step -- forward, loss, backward with the data-parallel reducer's bucket packs and RCCL
all-reduces on its comm stream, the fused optimizer update -- into one ``torch.cuda.CUDAGraph``
(a hipGraph on ROCm) and replays it.  Every kernel of the step still runs on every replay: the
graph changes how the work is launched, not what is computed.

Rules of the captured step (the usual whole-network capture rules): static input tensors (copy
new data into them), a constant learning rate (the fused optimizer bakes the hyper-parameters
into its kernel arguments), no host synchronisation inside the step (``nonfinite="ignore"``), and
the first steps -- bucket re-layout, per-shape kernel choices, MIOpen solver selection -- taken
eagerly during the warm-up before capture.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class CapturedStep:
    """A step recorded in a HIP graph; ``__call__`` replays it and returns the static output."""

    def __init__(self, graph, output, pool):
        self.graph, self.output, self.pool = graph, output, pool
        self.replays = 0

    def __call__(self):
        self.graph.replay()
        self.replays += 1
        return self.output


def capture_step(step: Callable[[], Optional[torch.Tensor]], warmup: int = 3) -> Optional[CapturedStep]:
    """Run ``step`` ``warmup`` times eagerly on a side stream, then capture one call of it.
    Returns None (run eagerly) without a GPU."""
    if not torch.cuda.is_available():
        return None
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(warmup):
            step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    pool = torch.cuda.graph_pool_handle()
    with torch.cuda.graph(g, pool=pool):
        out = step()
    torch.cuda.synchronize()
    return CapturedStep(g, out, pool)


def capturing() -> bool:
    """True while the current stream records a graph (callers skip timing events / host syncs)."""
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
