"""Job-start communication probe: the reference's ``comm_speed`` (datamodule.lua:280-303) made real.

The reference meant to time its synchronisation and feed the measured ``speed`` into
``optimize_sync`` (datamodule.lua:42,46,65); the call was commented out.  Here every multi-rank
``plan_model`` spends about a second measuring the job's OWN communicators before it prices
any placement:

* an all-reduce of a small message on the world group (the per-collective latency the
  bucket timeline adds per reduction) and of a large one (the bus bandwidth RCCL reaches
  over xGMI for gradient buckets);
* a pairwise bidirectional exchange between ranks (2i, 2i+1) as one ``batch_isend_irecv`` --
  exactly the pipeline transport's operation -- for the per-direction point-to-point rate.

Every timing is the MAX over ranks (all ranks see the same numbers and plan the same
placement).  :func:`apply` turns the result into the planner's :class:`~madnn.planner.hw.Machine`
(``allreduce_eff``, ``collective_latency_us``, ``p2p_gbps``) instead of the datasheet values.
"""
from __future__ import annotations

import os
import time
from dataclasses import replace
from typing import Optional

import torch
import torch.distributed as dist

from .. import runtime as rt


def _timed(fn, iters: int, group=None) -> float:
    """Seconds per call of ``fn`` (one warm-up call), MAX over the ranks of ``group``."""
    on_gpu = rt.device().type == "cuda" and torch.cuda.is_available()
    fn()
    if on_gpu:
        torch.cuda.synchronize()
    rt.barrier(group, monitored=False)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    if on_gpu:
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    nccl = dist.get_backend(group) == "nccl"
    t = torch.tensor([dt], dtype=torch.float64, device=rt.device() if nccl else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def measure(group=None, big_bytes: Optional[int] = None, small_bytes: int = 64 << 10,
            p2p_bytes: Optional[int] = None, iters: int = 3) -> dict:
    """Measure the all-reduce latency / bus bandwidth and the pairwise P2P rate of ``group``
    (default: the world).  Sizes default to 64 MiB / 16 MiB on RCCL and 4 MiB / 1 MiB on gloo,
    which keeps the probe near one second."""
    if not dist.is_initialized():
        return {}
    w = rt.get_world_size(group)
    if w < 2:
        return {}
    nccl = dist.get_backend(group) == "nccl"
    dev = rt.device() if nccl else torch.device("cpu")   # gloo: host tensors
    big = int(big_bytes or ((64 << 20) if nccl else (4 << 20)))
    p2pb = int(p2p_bytes or ((16 << 20) if nccl else (1 << 20)))
    dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
    esz = torch.tensor([], dtype=dt).element_size()
    out = {"world": w, "backend": dist.get_backend(group)}
    xs = torch.ones(max(small_bytes // esz, 1), dtype=dt, device=dev)
    t_small = _timed(lambda: dist.all_reduce(xs, group=group), iters, group)
    xb = torch.ones(big // esz, dtype=dt, device=dev)
    t_big = _timed(lambda: dist.all_reduce(xb, group=group), iters, group)
    out["allreduce_small_us"] = t_small * 1e6
    out["allreduce_bytes"] = xb.numel() * esz
    out["allreduce_busbw_gbps"] = 2.0 * (w - 1) / w * xb.numel() * esz / t_big / 1e9
    # pairwise exchange (2i <-> 2i+1) as one batch, the pipeline transport's operation
    ranks = dist.get_process_group_ranks(group) if group is not None else list(range(w))
    me = ranks.index(dist.get_rank())
    peer = me ^ 1
    a = torch.ones(p2pb // esz, dtype=dt, device=dev)
    b = torch.empty_like(a)

    def exchange():
        if peer < w:
            ops = [dist.P2POp(dist.isend, a, ranks[peer], group), dist.P2POp(dist.irecv, b, ranks[peer], group)]
            for work in dist.batch_isend_irecv(ops):
                work.wait()

    t_p2p = _timed(exchange, iters, group)
    out["p2p_bytes"] = a.numel() * esz
    out["p2p_gbps"] = a.numel() * esz / t_p2p / 1e9
    return out


def apply(machine, probe: dict):
    """A copy of ``machine`` with the measured link numbers: the all-reduce efficiency against
    the model's ring bound over min(links, W-1) xGMI links, the small-message latency, and the
    per-direction point-to-point rate."""
    if not probe:
        return machine
    w = int(probe["world"])
    ring = machine.link_gbps * max(min(machine.links, w - 1), 1)
    eff = min(max(probe["allreduce_busbw_gbps"] / ring, 0.01), 1.0)
    return replace(machine, allreduce_eff=eff, collective_latency_us=float(probe["allreduce_small_us"]),
                   p2p_gbps=float(probe["p2p_gbps"]),
                   calibrated=(machine.calibrated + "; " if machine.calibrated else "")
                   + f"comm measured at job start world={w} backend={probe['backend']}",
                   source=machine.source + "+comm-probe")


def wanted(cfg) -> bool:
    """``cfg.extra['measure_comm']`` / ``MADNN_PLAN_COMM`` (default on whenever W > 1)."""
    v = cfg.extra.get("measure_comm", os.environ.get("MADNN_PLAN_COMM", "1"))
    if isinstance(v, str):
        return v.lower() not in ("0", "false", "no", "off")
    return bool(v)
