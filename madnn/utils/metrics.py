"""Per-step training metrics: loss, samples/s, step time, the part of it the
compute stream spent waiting on gradient communication, the pipeline bubble, peak HBM,
all-reduce bytes and effective bus bandwidth -- one dict per step, optionally appended to a
JSONL file (``MetricsSink``).

    meter = StepMeter(engine, samples_per_step=B, path="metrics.jsonl")
    for x, y in loader:
        meter.start()
        loss = engine.train_step(x, y); opt.step()
        m = meter.stop(loss)          # {'step': .., 'step_ms': .., 'samples_per_s': .., ...}

The reference only prints the trainer error (datamodule.lua:173-175) and the shard ranges
(datamodule.lua:261).  Comm numbers come from HIP events the engines record themselves
(``DataParallel.comm_metrics``); ``stop`` synchronises the device once per step, so use it
for monitoring runs, not inside a timed benchmark loop.
"""
from __future__ import annotations

import time
from typing import Optional

import torch

from .logging import MetricsSink


class StepMeter:
    def __init__(self, engine=None, samples_per_step: Optional[int] = None, path: Optional[str] = None,
                 all_ranks: bool = False):
        self.engine = engine
        self.samples_per_step = samples_per_step
        self.sink = MetricsSink(path, all_ranks=all_ranks)
        self.step = 0
        self._t0 = None
        self.history = []

    def start(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self._t0 = time.perf_counter()

    def stop(self, loss=None, **extra) -> dict:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dt = time.perf_counter() - (self._t0 if self._t0 is not None else time.perf_counter())
        self.step += 1
        m = {"step": self.step, "step_ms": dt * 1e3}
        if loss is not None:
            m["loss"] = float(loss.detach()) if isinstance(loss, torch.Tensor) else float(loss)
        if self.samples_per_step and dt > 0:
            m["samples_per_s"] = self.samples_per_step / dt
        if self.engine is not None and hasattr(self.engine, "comm_metrics"):
            m.update(self.engine.comm_metrics())
        if torch.cuda.is_available():
            m["peak_hbm_gb"] = torch.cuda.max_memory_allocated() / 1e9
        m.update(extra)
        self.history.append(m)
        self.sink.log(**m)
        return m

    def close(self):
        self.sink.close()
