"""Fault injection for the failure-detection path.

``MADNN_FAULT=rank:step:kind`` makes ``maybe_fail(step)`` on that rank
``raise`` (exception), ``exit`` (hard exit 17) or ``hang`` (sleep forever) at
that step; ``corrupt`` instead poisons that rank's gradients of that step with
NaN before they are reduced (``maybe_corrupt``), which the optimizers'
``nonfinite`` guard must catch on every rank.  Tests use it to prove that the launcher tears the job down and
that process-group timeouts fire instead of deadlocking.  The reference has
no failure handling beyond MPI's default abort.
"""
from __future__ import annotations

import os
import time


class InjectedFault(RuntimeError):
    pass


def parse(spec: str):
    r, s, kind = spec.split(":")
    return int(r), int(s), kind


def maybe_fail(step: int, rank: int = None) -> None:
    spec = os.environ.get("MADNN_FAULT")
    if not spec:
        return
    r, s, kind = parse(spec)
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    if rank != r or step != s or kind == "corrupt":
        return
    if kind == "raise":
        raise InjectedFault(f"injected fault on rank {rank} at step {step}")
    if kind == "exit":
        os._exit(17)
    if kind == "hang":
        while True:
            time.sleep(3600)
    raise ValueError(f"unknown fault kind {kind!r}")


def maybe_corrupt(step: int, t, rank: int = None) -> bool:
    """Fill ``t`` with NaN when ``MADNN_FAULT`` names this rank, this step and kind ``corrupt``."""
    spec = os.environ.get("MADNN_FAULT")
    if not spec:
        return False
    r, s, kind = parse(spec)
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    if kind != "corrupt" or rank != r or step != s:
        return False
    t[:1].fill_(float("nan"))  # the first gradient element (bucket padding is never written)
    return True
