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


def enable_order_check(on: bool = True, every: Optional[int] = None) -> None:
    _checker["on"] = on
    _checker["hash"] = None
    if every is not None:
        _checker["every"] = int(every)


def order_check_enabled() -> bool:
    return _checker["on"]


def check_every() -> int:
    """Steps between two cross-rank fingerprint comparisons (``MADNN_CHECK_EVERY``, default 50)."""
    return _checker.get("every") or int(os.environ.get("MADNN_CHECK_EVERY", "50"))


def _record(op: str, group, t: Optional[torch.Tensor]):
    if not _checker["on"]:
        return
    if _checker["hash"] is None:
        from ..ops.native_runtime import OrderHash

        _checker["hash"] = OrderHash()
    gid = 0
    if _is_local_group(group):
        gid = hash(("local", group.rank)) & 0x7FFFFFFF
    elif group is not None and dist.is_initialized():
        gid = hash(tuple(dist.get_process_group_ranks(group))) & 0x7FFFFFFF
    numel = t.numel() if t is not None else 0
    dt = _DT.get(t.dtype, 9) if t is not None else 0
    _checker["hash"].add(_OPS[op], gid, numel, dt)


def order_fingerprint() -> tuple:
    h = _checker["hash"]
    return (0, 0) if h is None else (h.h, h.count)


def verify_order(group=None) -> bool:
    """All ranks compare their collective fingerprints; raises on divergence."""
    if not dist.is_initialized() or _is_local_group(group):
        return True
    mine = order_fingerprint()
    objs = [None] * dist.get_world_size(group)
    dist.all_gather_object(objs, mine, group=group)
    if any(o != objs[0] for o in objs):
        raise RuntimeError(f"madnn: collective order diverged across ranks: {objs}")
    return True


def _is_local_group(group) -> bool:
    from ..runtime import LocalGroup

    return isinstance(group, LocalGroup)


def device_kind(t: torch.Tensor) -> str:
    return "gpu" if t.device.type == "cuda" else "cpu"


class Selected:
    """What :func:`select` chose for one tensor: the bound collective, its mode and the path
    label ``(device kind, transport)`` -- ``("gpu", "rccl")``, ``("gpu", "xgmi-oneshot")``,
    ``("gpu", "gloo-host")`` or ``("cpu", "gloo")`` -- mirroring the reference's
    ``collectiveSelector[dev][topo][sync|async][op]`` table lookup (datamodule.lua:199-208).
    A ``sync`` selection returns when the result may be used (RCCL: stream-ordered); an
    ``async`` one returns a work handle whose ``wait()`` orders the consumer after it."""

    __slots__ = ("fn", "device", "transport", "op", "mode")

    def __init__(self, fn, device, transport, op, mode="sync"):
        self.fn, self.device, self.transport, self.op, self.mode = fn, device, transport, op, mode

    def __call__(self, *args, **kwargs):
        if self.mode == "async" and self.op not in ("send", "recv", "barrier"):
            kwargs.setdefault("async_op", True)
        return self.fn(*args, **kwargs)

    def __repr__(self):
        return f"Selected({self.op}, {self.mode}, {self.device}/{self.transport})"


def select(t: torch.Tensor, op: str, group=None, mode: str = "sync") -> Selected:
    """Collective selector (R9): the implementation for ``op`` on ``t`` over ``group``.

    The reference keys on [cpu|gpu][singlenode|multinode][sync|async][op]; on one MI355X node
    the topology axis collapses (all 8 GPUs are xGMI peers) and the transport follows from the
    tensor's device, the group's backend and the mode: HIP tensors on an RCCL ("nccl") group
    travel over xGMI -- small sync sums through the K5 one-shot kernel when registered, an
    async sum always through RCCL (the one-shot kernel is stream-ordered only); HIP tensors on
    a gloo group (several ranks sharing one GPU in tests) are staged through host memory by
    gloo; host tensors go to gloo.  A host tensor on an RCCL group is refused (RCCL cannot
    move it).  Without a process group the returned callable is the local no-op of every
    collective."""
    if op not in _OPS:
        raise KeyError(f"unknown collective {op!r}")
    if mode not in ("sync", "async"):
        raise KeyError(f"unknown collective mode {mode!r} (sync | async)")
    fn = {"all_reduce": all_reduce, "broadcast": broadcast, "all_gather": all_gather_into,
          "reduce_scatter": reduce_scatter, "send": send, "recv": recv, "barrier": None}[op]
    kind = device_kind(t)
    if not dist.is_initialized() or _is_local_group(group):
        return Selected(fn or (lambda *a, **k: None), kind, "local", op, mode)
    be = dist.get_backend(group)
    if kind == "cpu" and be == "nccl":
        raise RuntimeError("CPU tensor on an RCCL group: use a gloo group for host tensors")
    transport = "rccl" if be == "nccl" else ("gloo-host" if kind == "gpu" else "gloo")
    if op == "all_reduce" and kind == "gpu" and mode == "sync":
        from .oneshot import lookup

        if lookup(t, group) is not None:
            transport = "xgmi-oneshot"   # K5: small sums over P2P-mapped peer buffers
    if fn is None:
        from .. import runtime as rt

        fn = lambda *a, **k: rt.barrier(group)  # noqa: E731
    return Selected(fn, kind, transport, op, mode)


def selector_table(group=None) -> dict:
    """The whole selection table for ``group`` in the reference's shape,
    ``{dev: {topology: {sync|async: {op: transport}}}}`` (one node: topology ``singlenode``)."""
    out = {}
    devs = [("cpu", torch.zeros(1))]
    if torch.cuda.is_available():
        devs.append(("gpu", torch.zeros(1, device="cuda")))
    for dev, t in devs:
        modes = {}
        for mode in ("sync", "async"):
            row = {}
            for op in _OPS:
                try:
                    row[op] = select(t, op, group, mode).transport
                except RuntimeError:
                    row[op] = None
            modes[mode] = row
        out[dev] = {"singlenode": modes}
    return out


def _local(group) -> bool:
    """True when a collective over ``group`` needs no communication at all: there is no
    process group, or ``group`` is a singleton SUB-group of a larger world (e.g. the pp
    axis of a pure-DP mesh).  The WORLD group is never local, even at world size 1: a
    launched world-1 job (``torch.distributed.run --nproc-per-node 1``) issues its
    RCCL collectives exactly like the 8-GPU job does, so the communicator setup and
    the reducer's stream/event protocol run on the 1-GPU box too."""
    if not dist.is_initialized() or _is_local_group(group):
        return True
    return group is not None and group is not dist.group.WORLD and dist.get_world_size(group) == 1


def all_reduce(t: torch.Tensor, op: str = "sum", group=None, async_op: bool = False):
    if _local(group):
        return None
    _record("all_reduce", group, t)
    if op == "sum" and not async_op and t.device.type == "cuda":
        from .oneshot import lookup

        c = lookup(t, group)   # K5 one-shot (MADNN_ONESHOT=1, registered via oneshot.enable_for)
        if c is not None:
            c(t)
            return None
    rop = {"sum": dist.ReduceOp.SUM, "avg": dist.ReduceOp.AVG, "max": dist.ReduceOp.MAX}[op]
    if rop == dist.ReduceOp.AVG and dist.get_backend(group) == "gloo":
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=False)
        t.div_(dist.get_world_size(group))
        return None
    return dist.all_reduce(t, op=rop, group=group, async_op=async_op)


def broadcast(t: torch.Tensor, src: int = 0, group=None, async_op: bool = False):
    """Broadcast from global rank ``src`` (reference synchronizeParameters, datamodule.lua:33)."""
    if _local(group):
        return None
    _record("broadcast", group, t)
    return dist.broadcast(t, src=src, group=group, async_op=async_op)


def all_gather_into(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    """out = cat over ranks of inp along dim 0 (reference allgatherTensor, nodemodule.lua:166,266)."""
    if _local(group):
        out.copy_(inp.reshape(out.shape))
        return None
    _record("all_gather", group, inp)
    return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)


def reduce_scatter(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    if _local(group):
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


def all_agree(ok: bool, group=None) -> bool:
    """True on every rank iff ``ok`` is true on every rank of ``group`` (a MIN all-reduce).  Ranks
    call it after a step that may fail locally and BEFORE any collective that depends on it, so a
    local failure becomes a common decision instead of peers blocked in a gather."""
    if _local(group) or not dist.is_initialized():
        return bool(ok)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def log_backend_once():
    if dist.is_initialized():
        get_logger().info("comm backend=%s world=%d", dist.get_backend(), dist.get_world_size())
