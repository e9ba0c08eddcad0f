"""Hardware calibration: measure THIS node and persist the planner's machine profile.

    python -m madnn.planner.calibrate                       # 1 GPU: HBM + GEMM
    python -m madnn.launch --nproc 8 -m madnn.planner.calibrate   # + xGMI all-reduce / P2P

The reference meant to time forward/backward/sync (``comm_speed``,
datamodule.lua:280-303) and feed the result into its sync-period choice
(datamodule.lua:42,46) but never wired it.  Here the measured numbers replace
the datasheet defaults of :class:`~madnn.planner.hw.Machine`:

* ``hbm_tbps``       -- streaming copy bandwidth (read + write bytes / time);
* ``bf16_tflops``    -- a large bf16 GEMM on hipBLASLt (the rate GEMM-heavy layers see);
* ``fp32_tflops``    -- the same GEMM in fp32;
* ``link_gbps`` / ``allreduce_eff`` / ``p2p_gbps`` / ``collective_latency_us`` --
  from the all-reduce sweep and the P2P ping-pong when the job has > 1 rank.

The profile is written as JSON to ``path`` (default: :func:`hw.default_profile_path`),
which :func:`hw.load` reads by default, so every later ``distribute()`` on the node
plans with measured numbers without any flag.
"""
from __future__ import annotations

import argparse
import json
import time
from dataclasses import asdict
from typing import Optional

import torch
import torch.distributed as dist

from .. import runtime as rt
from .hw import Machine, default_profile_path, dump, invalidate


def _time_cuda(fn, iters: int = 10, warmup: int = 3) -> float:
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters / 1e3


def measure_hbm(nbytes: int = 2 << 30) -> float:
    """TB/s of a device-to-device copy (bytes read + bytes written)."""
    x = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    y = torch.empty_like(x)
    t = _time_cuda(lambda: y.copy_(x))
    return 2 * nbytes / t / 1e12


def measure_gemm(n: int = 8192, dtype=torch.bfloat16) -> float:
    a = torch.randn(n, n, device="cuda", dtype=dtype)
    b = torch.randn(n, n, device="cuda", dtype=dtype)
    t = _time_cuda(lambda: a @ b, iters=10)
    return 2.0 * n ** 3 / t / 1e12


def calibrate(path: Optional[str] = None, comm: bool = True, quick: bool = False) -> Machine:
    """Measure this node and write the profile (rank 0).  Collective when > 1 rank."""
    rt.init()
    m = Machine()
    if torch.cuda.is_available():
        m.name = torch.cuda.get_device_name()
        m.hbm_gb = torch.cuda.get_device_properties(0).total_memory / 1e9
        m.hbm_tbps = round(measure_hbm(1 << 30 if quick else 2 << 30), 3)
        m.bf16_tflops = round(measure_gemm(4096 if quick else 8192, torch.bfloat16), 1)
        m.fp32_tflops = round(measure_gemm(4096, torch.float32), 1)
    w = rt.get_world_size()
    if comm and w > 1:
        from ..comm.bench import run

        sizes = [1 << 12, 1 << 20, 64 << 20] if quick else [1 << 12, 1 << 16, 1 << 20, 16 << 20, 256 << 20]
        res = run(sizes, iters=10, warmup=3, ops=("all_reduce", "p2p"))
        small, big = res[0], res[-1]
        m.collective_latency_us = round(small["all_reduce_us"], 2)
        # busbw of the big all-reduce = per-GPU bandwidth RCCL spreads over min(links, W-1) links
        lanes = min(m.links, w - 1)
        m.allreduce_eff = 1.0
        m.link_gbps = round(big["all_reduce_busbw_gbps"] / lanes, 2)
        if "p2p_gbps" in big:
            m.p2p_gbps = round(big["p2p_gbps"], 2)
    m.calibrated = time.strftime("%Y-%m-%dT%H:%M:%S") + f" world={w}"
    if rt.get_rank() == 0:
        out = path or default_profile_path()
        dump(m, out)
        invalidate()
    if dist.is_initialized():
        rt.barrier()
    return m


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m madnn.planner.calibrate")
    ap.add_argument("--out", default=None)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--no-comm", action="store_true")
    a = ap.parse_args(argv)
    m = calibrate(a.out, comm=not a.no_comm, quick=a.quick)
    if rt.get_rank() == 0:
        print(json.dumps(asdict(m)))
    rt.shutdown()


if __name__ == "__main__":
    main()
