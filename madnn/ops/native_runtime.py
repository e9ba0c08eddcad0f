"""ctypes bindings for the host C++ runtime (``_madnn_runtime.so``).

Built from ``csrc/runtime.cpp`` with g++ (no GPU needed); if the library is
missing it is built on first use.  See runtime.cpp for the algorithms.
"""
from __future__ import annotations

import ctypes
import threading
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

HERE = Path(__file__).resolve().parent
_SO = HERE / "_madnn_runtime.so"
_lib = None
_lock = threading.Lock()


def _load():
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not _SO.exists():
            from .build import build

            build()
        lib = ctypes.CDLL(str(_SO))
        D, I, L, U = ctypes.c_double, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64
        lib.madnn_partition.restype = D
        lib.madnn_partition.argtypes = [ctypes.POINTER(D), ctypes.POINTER(D), I, I, D, ctypes.POINTER(I)]
        lib.madnn_plan_buckets.restype = I
        lib.madnn_plan_buckets.argtypes = [ctypes.POINTER(L), I, L, I, ctypes.POINTER(I), ctypes.POINTER(L),
                                           ctypes.POINTER(L)]
        lib.madnn_pipeline_order.restype = I
        lib.madnn_pipeline_order.argtypes = [I, I, I, I, I, ctypes.POINTER(I)]
        lib.madnn_hash_init.restype = U
        lib.madnn_hash_init.argtypes = []
        lib.madnn_hash_event.restype = U
        lib.madnn_hash_event.argtypes = [U, I, I, L, I]
        _lib = lib
        return lib


def partition(costs: Sequence[float], nstages: int, mems: Optional[Sequence[float]] = None,
              mem_cap: float = 0.0) -> Tuple[List[int], float]:
    """Contiguous partition of layers into ``nstages`` minimising the max stage cost.

    Returns (bounds, bottleneck) with bounds[0] = 0 and bounds[-1] = len(costs).
    Raises ValueError if no partition fits ``mem_cap``.
    """
    lib = _load()
    L = len(costs)
    c = (ctypes.c_double * L)(*costs)
    m = (ctypes.c_double * L)(*(mems if mems is not None else [0.0] * L))
    b = (ctypes.c_int * (nstages + 1))()
    best = lib.madnn_partition(c, m, L, nstages, float(mem_cap), b)
    if best < 0:
        raise ValueError(f"no {nstages}-stage partition of {L} layers fits mem_cap={mem_cap}")
    return list(b), best


def plan_buckets(numels: Sequence[int], cap_elems: int, align: int = 16):
    """Greedy bucket assignment in the given (backward-ready) order.

    Returns (bucket_of, offset_of, bucket_sizes).
    """
    lib = _load()
    n = len(numels)
    ne = (ctypes.c_int64 * max(n, 1))(*numels)
    bo = (ctypes.c_int * max(n, 1))()
    oo = (ctypes.c_int64 * max(n, 1))()
    bs = (ctypes.c_int64 * max(n, 1))()
    nb = lib.madnn_plan_buckets(ne, n, int(max(cap_elems, 1)), int(align), bo, oo, bs)
    return list(bo)[:n], list(oo)[:n], list(bs)[:nb]


SCHEDULE_KINDS = {"gpipe": 0, "1f1b": 1, "interleaved": 2}


def pipeline_order(kind: str, stage: int, nstages: int, nmicro: int, nchunks: int = 1) -> List[Tuple[str, int, int]]:
    """Per-rank compute order [("F"|"B", chunk, microbatch)] of a pipeline schedule
    (GPipe, 1F1B, or interleaved 1F1B with ``nchunks`` model chunks per rank)."""
    lib = _load()
    if kind not in SCHEDULE_KINDS:
        raise ValueError(f"unknown pipeline schedule {kind!r}")
    n = 2 * nmicro * nchunks
    out = (ctypes.c_int * (3 * n + 3))()
    k = lib.madnn_pipeline_order(SCHEDULE_KINDS[kind], stage, nstages, nmicro, nchunks, out)
    if k < 0:
        raise ValueError(f"invalid pipeline order: kind={kind} stage={stage}/{nstages} microbatches={nmicro} "
                         f"chunks={nchunks} (interleaved needs microbatches % stages == 0; gpipe/1f1b one chunk)")
    vals = list(out)[:3 * k]
    return [("F" if vals[3 * i] == 0 else "B", vals[3 * i + 1], vals[3 * i + 2]) for i in range(k)]


class OrderHash:
    """Rolling fingerprint of the collective sequence issued by this rank."""

    def __init__(self):
        self.lib = _load()
        self.h = self.lib.madnn_hash_init()
        self.count = 0

    def add(self, op: int, group: int, numel: int, dtype: int) -> None:
        self.h = self.lib.madnn_hash_event(self.h, op, group, numel, dtype)
        self.count += 1
