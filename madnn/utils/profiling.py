"""Step-timeline profiling: ``torch.profiler`` with its ROCm backend (roctracer)
records host ops, HIP kernel launches and kernels, so a training loop's overlap -- bucket
all-reduces on the comm stream under backward, pipeline sends under compute -- is visible on a
timeline.  Kernel-level counters stay with rocprofv3 (``scripts/gpu_*pmc*.sh``); this is the
in-process view.

    with madnn.utils.profiling.step_profiler("gpurun_out/trace", active=3) as prof:
        for _ in range(6):
            train_step(); prof.step()

writes one Chrome/Perfetto trace per rank (``trace-rank<r>.json``) and returns the profiler, whose
``key_averages()`` table can be printed too.
"""
from __future__ import annotations

import os
from contextlib import contextmanager

import torch


@contextmanager
def step_profiler(out_dir: str, wait: int = 1, warmup: int = 1, active: int = 3, record_shapes: bool = False):
    """A ``torch.profiler.profile`` over ``wait + warmup + active`` steps (call ``prof.step()``
    once per training step) that writes this rank's trace to ``out_dir/trace-rank<r>.json``."""
    from torch.profiler import ProfilerActivity, profile, schedule

    from .. import runtime as rt

    os.makedirs(out_dir, exist_ok=True)
    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)  # HIP kernels through roctracer on ROCm
    path = os.path.join(out_dir, f"trace-rank{rt.get_rank()}.json")

    def on_ready(p):
        p.export_chrome_trace(path)

    with profile(activities=acts, schedule=schedule(wait=wait, warmup=warmup, active=active),
                 on_trace_ready=on_ready, record_shapes=record_shapes) as prof:
        yield prof


def kernel_table(prof, n: int = 20) -> str:
    """The ``n`` most expensive ops / kernels of a finished profile, by device time when a GPU
    was profiled."""
    key = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
    return prof.key_averages().table(sort_by=key, row_limit=n)
