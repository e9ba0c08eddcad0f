"""Rank-aware logging and a JSONL metrics sink.

The reference only ``print``s (shard ranges, datamodule.lua:261; comm speed,
datamodule.lua:300; trainer error, datamodule.lua:173-175).  Here every
message carries the rank, rank 0 logs by default and ``MADNN_LOG_ALL_RANKS=1``
opens the other ranks.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time

_LOGGER = None


def _rank() -> int:
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:
        pass
    return int(os.environ.get("RANK", "0"))


class _RankFilter(logging.Filter):
    def filter(self, record: logging.LogRecord) -> bool:
        record.rank = _rank()
        if os.environ.get("MADNN_LOG_ALL_RANKS", "0") == "1":
            return True
        return record.rank == 0 or record.levelno >= logging.WARNING


def get_logger() -> logging.Logger:
    global _LOGGER
    if _LOGGER is None:
        log = logging.getLogger("madnn")
        if not log.handlers:
            h = logging.StreamHandler(sys.stderr)
            h.setFormatter(logging.Formatter("[madnn r%(rank)s %(levelname)s] %(message)s"))
            h.addFilter(_RankFilter())
            log.addHandler(h)
        log.setLevel(os.environ.get("MADNN_LOG_LEVEL", "INFO").upper())
        log.propagate = False
        _LOGGER = log
    return _LOGGER


class MetricsSink:
    """Append-only JSONL metrics (one dict per step), rank 0 only by default."""

    def __init__(self, path: str | None, all_ranks: bool = False):
        self.path = path
        self.enabled = path is not None and (all_ranks or _rank() == 0)
        self._fh = open(path, "a") if self.enabled else None

    def log(self, **kv):
        if not self._fh:
            return
        kv.setdefault("ts", time.time())
        kv.setdefault("rank", _rank())
        self._fh.write(json.dumps(kv) + "\n")
        self._fh.flush()

    def close(self):
        if self._fh:
            self._fh.close()
            self._fh = None
