"""K5: one-shot all-reduce over P2P-mapped peer buffers (``madnn/ops/csrc/xgmi.hip``).

For the small, latency-bound all-reduces of tensor parallelism (the reference's MP layers sum
``[B, out]`` activation shards every layer, ``/root/reference/nodemodule.lua:52,103``).  Every
rank allocates a staging buffer and an uncached flag array, the IPC handles are exchanged once
over the process group, and each call is ONE kernel per rank: stage the input, raise a flag in
every peer, wait for the peers' flags, sum the W staged inputs read straight over xGMI.

    comm = OneShotAllReduce(group, cap_bytes=8 << 20)
    comm(t)                      # in-place sum over the group (fp32 or bf16 HIP tensor)
    comm.check()                 # synchronise; raise if a peer never arrived (bounded wait)

A wait that times out leaves this rank's own input in the output, so the error must be loud: the
kernel records it in a pinned host word that every later call (and :func:`poll_all`, run by the
engines' per-step robustness hook) reads without synchronising, raising ``OneShotTimeout`` at
the latest one optimizer step after the failed call.

``madnn.comm.all_reduce`` routes small HIP tensors through a registered communicator when
``MADNN_ONESHOT=1`` (:func:`enable_for`); RCCL stays the default until the one-shot path is
measured against it on an 8-GPU node.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch
import torch.distributed as dist

_lib = {"h": None}
_registry: dict = {}


def _native():
    if _lib["h"] is None:
        from .. import ops

        if not ops.load_kernels():
            raise RuntimeError("madnn: the HIP kernel library is needed for the one-shot all-reduce")
        lib = ctypes.CDLL(str(ops.kernels_path()))
        I, L, P = ctypes.c_int, ctypes.c_int64, ctypes.c_void_p
        lib.madnn_oneshot_create.argtypes = [L, I, I, I, P]
        lib.madnn_oneshot_create.restype = I
        lib.madnn_oneshot_open.argtypes = [I, P]
        lib.madnn_oneshot_open.restype = I
        lib.madnn_oneshot_allreduce.argtypes = [I, P, P, L, I, I, P]
        lib.madnn_oneshot_allreduce.restype = I
        lib.madnn_oneshot_error.argtypes = [I, I]
        lib.madnn_oneshot_error.restype = I
        lib.madnn_oneshot_destroy.argtypes = [I]
        lib.madnn_oneshot_destroy.restype = I
        lib.madnn_oneshot_handle_bytes.restype = I
        lib.madnn_oneshot_max_peers.restype = I
        _lib["h"] = lib
    return _lib["h"]


class OneShotTimeout(RuntimeError):
    pass


class OneShotAllReduce:
    """One-shot sum all-reduce over ``group`` (all ranks on this node, <= 8)."""

    def __init__(self, group=None, cap_bytes: int = 8 << 20, spin_limit: int = 1 << 21,
                 device: Optional[torch.device] = None):
        lib = _native()
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if self.world > lib.madnn_oneshot_max_peers():
            raise ValueError(f"one-shot all-reduce spans at most {lib.madnn_oneshot_max_peers()} ranks")
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.cap = int(cap_bytes)
        self.spin_limit = int(spin_limit)
        hb = lib.madnn_oneshot_handle_bytes()
        mine = (ctypes.c_ubyte * (2 * hb))()
        with torch.cuda.device(dev):
            cid = lib.madnn_oneshot_create(self.cap, self.world, self.rank, dev.index, mine)
        if cid <= 0:
            raise RuntimeError(f"madnn_oneshot_create failed (hipError {-cid})")
        self.id = cid
        handles = [bytes(mine)]
        if self.world > 1:
            handles = [None] * self.world
            dist.all_gather_object(handles, bytes(mine), group=group)
        allh = (ctypes.c_ubyte * (2 * hb * self.world)).from_buffer_copy(b"".join(handles))
        with torch.cuda.device(dev):
            rc = lib.madnn_oneshot_open(self.id, allh)
        if rc != 0:
            lib.madnn_oneshot_destroy(self.id)
            raise RuntimeError(f"madnn_oneshot_open failed (hipError {rc})")
        if self.world > 1:  # every rank mapped every peer before anyone writes a flag
            dist.barrier(group=group)

    def supports(self, t: torch.Tensor) -> bool:
        return (t.device == self.device and t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous()
                and t.numel() * t.element_size() <= self.cap)

    def __call__(self, t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if not self.supports(t):
            raise ValueError("one-shot all-reduce: contiguous fp32/bf16 tensor on this device within cap")
        self.poll()
        out = t if out is None else out
        stream = torch.cuda.current_stream(self.device).cuda_stream
        rc = _native().madnn_oneshot_allreduce(self.id, t.data_ptr(), out.data_ptr(), t.numel(),
                                               0 if t.dtype == torch.float32 else 1, self.spin_limit, stream)
        if rc != 0:
            raise RuntimeError(f"madnn_oneshot_allreduce failed (hipError {rc})")
        return out

    def _raise_if(self, err: int) -> None:
        if err != 0:
            raise OneShotTimeout("one-shot all-reduce: a peer never published its input within the bounded "
                                 "wait; the affected output holds only this rank's partial sum"
                                 if err > 0 else "one-shot all-reduce: error word unreadable")

    def poll(self) -> None:
        """Raise if a FINISHED call's wait timed out (host read of the pinned error word, no sync)."""
        if getattr(self, "id", 0) > 0:
            self._raise_if(_native().madnn_oneshot_error(self.id, 1))

    def check(self) -> None:
        """Synchronise and raise if any call's wait for a peer timed out since the last check."""
        self._raise_if(_native().madnn_oneshot_error(self.id, 3))

    def close(self) -> None:
        if getattr(self, "id", 0) > 0:
            _native().madnn_oneshot_destroy(self.id)
            self.id = 0


def enable_for(group=None, cap_bytes: int = 1 << 20) -> Optional[OneShotAllReduce]:
    """Register a one-shot communicator for ``group``: with ``MADNN_ONESHOT=1``,
    :func:`madnn.comm.all_reduce` sends sum all-reduces of HIP tensors up to ``cap_bytes`` through
    it (collective: every rank of the group must call this)."""
    if not (dist.is_initialized() and torch.cuda.is_available()):
        return None   # (any backend: the group only carries the one-time IPC handle exchange)
    c = OneShotAllReduce(group, cap_bytes=cap_bytes)
    _registry[_key(group)] = c
    return c


def poll_all() -> None:
    """Lazy error check of every registered communicator (engines call it once per step)."""
    for c in list(_registry.values()):
        c.poll()


def _key(group):
    return tuple(dist.get_process_group_ranks(group)) if group is not None else ("world",)


def lookup(t: torch.Tensor, group=None) -> Optional[OneShotAllReduce]:
    if not _registry or os.environ.get("MADNN_ONESHOT", "0") != "1":
        return None
    c = _registry.get(_key(group))
    return c if c is not None and c.supports(t) else None
