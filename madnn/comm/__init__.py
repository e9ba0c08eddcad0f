"""Collective layer: selector, instrumented collectives, order checker.

Reference: ``datamodule.selectCollective`` (datamodule.lua:199-208) picks a
TorchMPI implementation by device (cpu|gpu) and topology (singlenode|
multinode) from ``mpi.collectiveSelector``.  Here device tensors go to RCCL
(torch.distributed backend "nccl" on ROCm; xGMI inside the node) and CPU
tensors to gloo; the selector returns the backend-bound callable so callers
never issue a collective on the wrong backend.  Every collective can be
fingerprinted (op, group, numel, dtype) by the C++ OrderHash; ranks compare
fingerprints to catch the schedule divergence that otherwise deadlocks
(SURVEY §5.2).
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch
import torch.distributed as dist

from ..utils.logging import get_logger

_OPS = {"all_reduce": 1, "broadcast": 2, "all_gather": 3, "reduce_scatter": 4, "send": 5, "recv": 6, "barrier": 7}
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
_checker = {"on": os.environ.get("MADNN_CHECK_COLLECTIVES", "0") == "1", "hash": None}


def enable_order_check(on: bool = True) -> None:
    _checker["on"] = on
    _checker["hash"] = None


def _record(op: str, group, t: Optional[torch.Tensor]):
    if not _checker["on"]:
        return
    if _checker["hash"] is None:
        from ..ops.native_runtime import OrderHash

        _checker["hash"] = OrderHash()
    gid = 0
    if group is not None and dist.is_initialized():
        gid = hash(tuple(dist.get_process_group_ranks(group))) & 0x7FFFFFFF
    numel = t.numel() if t is not None else 0
    dt = _DT.get(t.dtype, 9) if t is not None else 0
    _checker["hash"].add(_OPS[op], gid, numel, dt)


def order_fingerprint() -> tuple:
    h = _checker["hash"]
    return (0, 0) if h is None else (h.h, h.count)


def verify_order(group=None) -> bool:
    """All ranks compare their collective fingerprints; raises on divergence."""
    if not dist.is_initialized():
        return True
    mine = order_fingerprint()
    objs = [None] * dist.get_world_size(group)
    dist.all_gather_object(objs, mine, group=group)
    if any(o != objs[0] for o in objs):
        raise RuntimeError(f"madnn: collective order diverged across ranks: {objs}")
    return True


def device_kind(t: torch.Tensor) -> str:
    return "gpu" if t.device.type == "cuda" else "cpu"


def select(t: torch.Tensor, op: str, group=None) -> Callable:
    """Collective selector (R9): returns a callable bound to the right backend.

    The reference keys on [cpu|gpu][singlenode|multinode][sync][op]; on a single
    MI355X node the topology axis collapses (all peers are xGMI), and the
    backend is fixed by the tensor's device.
    """
    if op not in _OPS:
        raise KeyError(f"unknown collective {op!r}")
    if not dist.is_initialized():
        return lambda *a, **k: None
    be = dist.get_backend(group)
    kind = device_kind(t)
    if kind == "gpu" and be not in ("nccl",):
        raise RuntimeError(f"device tensor on backend {be}: madnn routes HIP tensors to RCCL ('nccl')")
    if kind == "cpu" and be == "nccl":
        raise RuntimeError("CPU tensor on an RCCL group: use a gloo group for host tensors")
    fn = {"all_reduce": all_reduce, "broadcast": broadcast, "all_gather": all_gather_into,
          "reduce_scatter": reduce_scatter, "send": send, "recv": recv}.get(op)
    return fn


def all_reduce(t: torch.Tensor, op: str = "sum", group=None, async_op: bool = False):
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return None
    _record("all_reduce", group, t)
    rop = {"sum": dist.ReduceOp.SUM, "avg": dist.ReduceOp.AVG, "max": dist.ReduceOp.MAX}[op]
    if rop == dist.ReduceOp.AVG and dist.get_backend(group) == "gloo":
        w = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=False)
        t.div_(dist.get_world_size(group))
        return None
    return dist.all_reduce(t, op=rop, group=group, async_op=async_op)


def broadcast(t: torch.Tensor, src: int = 0, group=None, async_op: bool = False):
    """Broadcast from global rank ``src`` (reference synchronizeParameters, datamodule.lua:33)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return None
    _record("broadcast", group, t)
    return dist.broadcast(t, src=src, group=group, async_op=async_op)


def all_gather_into(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    """out = cat over ranks of inp along dim 0 (reference allgatherTensor, nodemodule.lua:166,266)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        out.copy_(inp.reshape(out.shape))
        return None
    _record("all_gather", group, inp)
    return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)


def reduce_scatter(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        out.copy_(inp.reshape(out.shape))
        return None
    _record("reduce_scatter", group, inp)
    return dist.reduce_scatter_tensor(out, inp, group=group, async_op=async_op)


def send(t: torch.Tensor, dst: int, group=None):
    _record("send", group, t)
    return dist.isend(t, dst, group=group)


def recv(t: torch.Tensor, src: int, group=None):
    _record("recv", group, t)
    return dist.irecv(t, src, group=group)


def log_backend_once():
    if dist.is_initialized():
        get_logger().info("comm backend=%s world=%d", dist.get_backend(), dist.get_world_size())
