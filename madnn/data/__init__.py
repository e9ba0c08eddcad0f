"""Data partitioning, synthetic datasets and a device-prefetching loader.

Reference: ``datamodule.data_parallel`` (datamodule.lua:235-267) gives rank r
the contiguous stripe ``[r*stripe, (r+1)*stripe)`` with
``stripe = floor(N / W)`` as a *view* of a dataset every rank loaded in full;
the remainder ``N mod W`` is dropped despite the comment claiming the last rank
gets it (SURVEY A-7), and an optional strided "shuffle" branch is disabled
(``dataShuffle=false``, datamodule.lua:3).  Here ``shard`` reproduces the
contiguous striping exactly (views, no copy) and makes the remainder policy
explicit: ``drop`` (reference behaviour, equal step counts), ``last`` (the
documented intent) or ``pad`` (wrap-around so every sample is seen).
"""
from __future__ import annotations

import math
from collections.abc import Mapping
from typing import Iterator, Optional, Sequence, Tuple

import torch

from .. import runtime as rt
from ..utils.logging import get_logger


_last_local = {"size": None}


def last_local_size() -> Optional[int]:
    """Samples in the shard this rank was last given by :func:`shard` or a
    :class:`DistributedSampler` (None if neither ran).  The reference sizes its sync period from
    the shard ``parallelize`` just cut (datamodule.lua:37-47); ``distribute(sync="params")`` reads
    it here when ``Config.local_size`` is not given."""
    return _last_local["size"]


def shard_bounds(n: int, rank: int, world: int, remainder: str = "drop") -> Tuple[int, int]:
    stripe = n // world
    start = rank * stripe
    end = start + stripe
    if remainder == "last" and rank == world - 1:
        end = n
    return start, end


def shard(data, rank: Optional[int] = None, world: Optional[int] = None, remainder: str = "drop",
          strided: bool = False, verbose: bool = False):
    """Rank's shard of ``data`` along dim 0 (tensor, list or any sliceable).

    ``strided=True`` is the reference's optional shuffle branch: rank r takes
    samples r, r+W, r+2W, ... (the reference wrote these through the view into
    the source tensor; this returns an index-select copy instead).
    """
    rank = rt.get_rank() if rank is None else rank
    world = rt.get_world_size() if world is None else world
    n = len(data)
    if strided:
        stripe = n // world
        idx = torch.arange(stripe) * world + rank  # empty when n < world (arange(rank, 0, W) would raise)
        out = data[idx] if isinstance(data, torch.Tensor) else [data[i] for i in idx.tolist()]
        if verbose:
            get_logger().info("rank %d: strided shard stripe=%d", rank, stripe)
        _last_local["size"] = len(out)
        return out
    start, end = shard_bounds(n, rank, world, remainder)
    if remainder == "pad":
        per = math.ceil(n / world)
        idx = [(rank * per + i) % n for i in range(per)]
        _last_local["size"] = per
        if isinstance(data, torch.Tensor):
            return data[torch.tensor(idx)]
        return [data[i] for i in idx]
    if verbose:
        get_logger().info("rank %d: shard [%d, %d) stripe=%d remainder=%d", rank, start, end, n // world,
                          n - (n // world) * world)
    _last_local["size"] = end - start
    return data[start:end]


class SyntheticImages(torch.utils.data.Dataset):
    """Deterministic random images + labels (no network on the GPU box)."""

    def __init__(self, n: int, shape=(3, 224, 224), num_classes: int = 1000, seed: int = 0):
        self.n, self.shape, self.num_classes, self.seed = n, tuple(shape), num_classes, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        return torch.randn(self.shape, generator=g), int(torch.randint(self.num_classes, (1,), generator=g))


class SyntheticTokens(torch.utils.data.Dataset):
    def __init__(self, n: int, seq_len: int, vocab: int, seed: int = 0):
        self.n, self.seq_len, self.vocab, self.seed = n, seq_len, vocab, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        return torch.randint(self.vocab, (self.seq_len,), generator=g)


def synthetic_batch(kind: str, batch: int, device, dtype=torch.bfloat16, **kw):
    """A device-resident synthetic batch generated ON the device (no H2D copy)."""
    g = torch.Generator(device=device).manual_seed(kw.get("seed", 1234))
    if kind == "image":
        c, h, w = kw.get("shape", (3, 224, 224))
        x = torch.randn(batch, c, h, w, device=device, generator=g, dtype=torch.float32).to(dtype)
        if kw.get("channels_last", False):
            x = x.contiguous(memory_format=torch.channels_last)
        y = torch.randint(kw.get("num_classes", 1000), (batch,), device=device, generator=g)
        return x, y
    if kind == "tokens":
        s, v = kw["seq_len"], kw["vocab"]
        ids = torch.randint(v, (batch, s), device=device, generator=g)
        return ids, ids
    raise ValueError(kind)


class DistributedSampler(torch.utils.data.Sampler):
    """Contiguous-stripe sampler with per-epoch shuffling inside the shard.

    Resumable: after :meth:`load_state_dict` the next iteration continues mid-epoch exactly
    where the saved one stopped (same permutation: it is a function of seed + epoch only).
    Restored at a different world size the position is carried over in GLOBAL samples.

    What is saved is the number of samples the TRAINING LOOP consumed this epoch, not the
    indices handed out: a DataLoader with workers, or madnn's :class:`DevicePrefetcher`, pulls
    batches ahead of the one being trained on, and saving the hand-out position would skip
    those on resume.  Iterate through :meth:`track` (it counts a batch when it reaches the loop)
    or call :meth:`advance` after each step; without either, the hand-out position is saved."""

    def __init__(self, n: int, rank: Optional[int] = None, world: Optional[int] = None, shuffle: bool = True,
                 remainder: str = "drop", seed: int = 0):
        self.n = n
        self.rank = rt.get_rank() if rank is None else rank
        self.world = rt.get_world_size() if world is None else world
        self.shuffle, self.remainder, self.seed = shuffle, remainder, seed
        self.epoch = 0
        self.cursor = 0          # indices of this epoch already yielded (may run ahead of training)
        self.consumed = 0        # samples of this epoch the training loop has taken (track / advance)
        self._tracked = False
        _last_local["size"] = len(self)

    def set_epoch(self, e: int):
        if e != self.epoch:
            self.cursor = 0
            self.consumed = 0
        self.epoch = e

    def advance(self, n: int) -> None:
        """The training loop finished ``n`` more samples of this epoch."""
        self._tracked = True
        self.consumed += int(n)

    def track(self, batches, batch_size: Optional[int] = None):
        """Yield from ``batches`` (a DataLoader / DevicePrefetcher over this sampler), counting
        each batch as consumed when it reaches the caller: a checkpoint taken in the loop body
        after the step resumes at the next unseen batch, however far the loader prefetched.

        A batch's size is read from its first tensor: element 0 of a list / tuple, the first value
        of a dict (HF-style collators), or the batch itself; any other batch type needs
        ``batch_size``."""
        self._tracked = True
        for b in batches:
            self.consumed += batch_size if batch_size is not None else _batch_len(b)
            yield b

    def position(self) -> int:
        """The resume position: consumed samples when the loop reports them, else handed out."""
        return min(self.consumed, self.cursor) if self._tracked else self.cursor

    def state_dict(self) -> dict:
        return {"n": self.n, "epoch": self.epoch, "cursor": self.position(), "seed": self.seed, "world": self.world,
                "shuffle": self.shuffle, "remainder": self.remainder}

    def load_state_dict(self, sd: dict) -> None:
        if int(sd["n"]) != self.n:
            raise ValueError(f"sampler state is for a dataset of {sd['n']} samples, not {self.n}")
        self.epoch, self.seed = int(sd["epoch"]), int(sd["seed"])
        cur = int(sd["cursor"])
        if int(sd.get("world", self.world)) != self.world:
            cur = cur * int(sd["world"]) // self.world   # same global position
        self.cursor = min(cur, len(self))
        self.consumed = self.cursor

    def _indices(self):
        if self.remainder == "pad":
            per = math.ceil(self.n / self.world)
            return [(self.rank * per + i) % self.n for i in range(per)]
        s, e = shard_bounds(self.n, self.rank, self.world, self.remainder)
        return list(range(s, e))

    def __iter__(self) -> Iterator[int]:
        idx = self._indices()
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            perm = torch.randperm(len(idx), generator=g).tolist()
            idx = [idx[i] for i in perm]
        start = self.cursor if self.cursor < len(idx) else 0
        self.cursor = start
        for i in idx[start:]:
            self.cursor += 1
            yield i

    def __len__(self):
        return len(self._indices())


def _batch_len(b) -> int:
    if isinstance(b, Mapping):
        if not b:
            raise ValueError("DistributedSampler.track: empty dict batch; pass batch_size=")
        b = next(iter(b.values()))
    elif isinstance(b, (list, tuple)):
        if not b:
            raise ValueError("DistributedSampler.track: empty batch; pass batch_size=")
        b = b[0]
    if isinstance(b, torch.Tensor):
        if b.dim() == 0:
            raise ValueError("DistributedSampler.track: 0-d batch tensor; pass batch_size=")
        return int(b.shape[0])
    if isinstance(b, (list, tuple)):
        return len(b)
    raise TypeError(f"DistributedSampler.track cannot size a {type(b).__name__} batch; pass batch_size=")


class DevicePrefetcher:
    """Overlaps the H2D copy of batch i+1 with compute on batch i (side HIP stream)."""

    def __init__(self, loader, device, dtype: Optional[torch.dtype] = None, channels_last: bool = False):
        self.loader, self.device, self.dtype, self.cl = loader, torch.device(device), dtype, channels_last
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None

    def _move(self, batch):
        if isinstance(batch, (list, tuple)):
            return type(batch)(self._move(b) for b in batch)
        if isinstance(batch, torch.Tensor):
            t = batch.to(self.device, non_blocking=True)
            if self.dtype is not None and t.is_floating_point():
                t = t.to(self.dtype)
            if self.cl and t.dim() == 4:
                t = t.contiguous(memory_format=torch.channels_last)
            return t
        return batch

    def __iter__(self):
        it = iter(self.loader)
        if self.stream is None:
            for b in it:
                yield self._move(b)
            return
        nxt = None
        try:
            with torch.cuda.stream(self.stream):
                nxt = self._move(next(it))
        except StopIteration:
            return
        while nxt is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            cur = nxt
            _record(cur, torch.cuda.current_stream(self.device))
            try:
                with torch.cuda.stream(self.stream):
                    nxt = self._move(next(it))
            except StopIteration:
                nxt = None
            yield cur


def _record(b, stream):
    if isinstance(b, torch.Tensor):
        b.record_stream(stream)
    elif isinstance(b, (list, tuple)):
        for x in b:
            _record(x, stream)
