"""Fault injection for the failure-detection path.

``MADNN_FAULT=rank:step:kind`` makes ``maybe_fail(step)`` on that rank
``raise`` (exception), ``exit`` (hard exit 17) or ``hang`` (sleep forever) at
that step.  Tests use it to prove that the launcher tears the job down and
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
    if rank != r or step != s:
        return
    if kind == "raise":
        raise InjectedFault(f"injected fault on rank {rank} at step {step}")
    if kind == "exit":
        os._exit(17)
    if kind == "hang":
        while True:
            time.sleep(3600)
    raise ValueError(f"unknown fault kind {kind!r}")
