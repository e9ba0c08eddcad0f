"""Process/device runtime: the ``mpi.start(true)`` equivalent.

Reference: ``mpi.start(true)`` (datamodule.lua:27; README.md:34,86) starts MPI,
binds a GPU and creates the communicator; ``mpi.rank()/size()/barrier()`` are
used throughout.  MI355X-native replacement: one process per GPU,
``torch.distributed`` with backend ``"nccl"`` (= RCCL over xGMI on ROCm) for
device tensors and ``gloo`` for CPU runs, plus named sub-groups for the
dp / pp / tp axes of a hybrid layout (the reference has a single world
communicator, which is why its DP and MP cannot be combined — SURVEY A-15).
"""
from __future__ import annotations

import datetime
import os
import random
import subprocess
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..utils.logging import get_logger

_STATE = {"initialized": False, "device": None, "backend": None}


def is_initialized() -> bool:
    return _STATE["initialized"]


def launched() -> bool:
    """True when a launcher (``torch.distributed.run``, ``madnn.launch``, bench.py) set up a
    rendezvous environment: RANK, WORLD_SIZE and MASTER_ADDR are all present."""
    return all(k in os.environ for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR"))


def init(backend: Optional[str] = None, timeout_s: float = 600.0, device: Optional[str] = None) -> None:
    """Bind this process to its GPU and join the process group (idempotent).

    Reads the torchrun / ``madnn.launch`` environment (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR, MASTER_PORT).  Under a launcher the process group
    is created even for a world of ONE, so the RCCL communicator setup, the
    reducer's all-reduce/broadcast and the device barrier run exactly as they do
    at 8 GPUs (``torch.distributed.run --nproc-per-node 1`` is the 1-GPU rehearsal
    of the 8-GPU path).  A plain ``python script.py`` without a launcher
    environment is a world of one with no process group.
    """
    if _STATE["initialized"]:
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and device != "cpu"
    if use_gpu:
        from ..utils.miopen import setup_find_db

        setup_find_db()  # shipped MI355X MIOpen find-db: tuned conv solvers without a search
        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    backend = backend or ("nccl" if use_gpu else "gloo")
    if (world > 1 or launched()) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev  # eager RCCL communicator init bound to this GPU
        dist.init_process_group(**kw)
    elif dist.is_initialized():
        backend = dist.get_backend()
    _STATE.update(initialized=True, device=dev, backend=backend)
    get_logger().debug("madnn.init rank=%d world=%d device=%s backend=%s", rank, world, dev, backend)


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
    _STATE.update(initialized=False, device=None, backend=None)
    ProcessGroups._cache.clear()


class LocalGroup:
    """A mesh axis of size ONE inside a larger world (the tp and cp axes of a dp x pp layout, the
    dp axis of a pure pipeline).  Every collective over it is the identity, so madnn creates no
    process group for it: an eagerly initialised RCCL communicator would bring its own HIP stream
    (and a share of the GPU's hardware queues) for nothing.  ``comm`` and this module treat it
    as a world of one in which this rank is rank 0."""

    __slots__ = ("rank",)

    def __init__(self, rank: int):
        self.rank = rank

    def __repr__(self):
        return f"LocalGroup(rank={self.rank})"


def is_local_group(group) -> bool:
    return isinstance(group, LocalGroup)


def get_rank(group=None) -> int:
    if isinstance(group, LocalGroup):
        return 0
    return dist.get_rank(group) if dist.is_initialized() else 0


def get_world_size(group=None) -> int:
    if isinstance(group, LocalGroup):
        return 1
    return dist.get_world_size(group) if dist.is_initialized() else 1


def get_local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def device() -> torch.device:
    if _STATE["device"] is None:
        init()
    return _STATE["device"]


def backend() -> str:
    if _STATE["backend"] is None:
        init()
    return _STATE["backend"]


def barrier(group=None, monitored: Optional[bool] = None, timeout_s: Optional[float] = None) -> None:
    """Global barrier (reference ``mpi.barrier()``, datamodule.lua:50).

    RCCL groups barrier on this rank's device.  gloo groups use
    ``monitored_barrier``: a rank that never arrives is NAMED in
    the error raised on rank 0 instead of every rank hanging silently.  Set
    ``monitored=False`` (or ``MADNN_MONITORED_BARRIER=0``) for a plain barrier."""
    if not dist.is_initialized() or isinstance(group, LocalGroup):
        return
    be = dist.get_backend(group)
    if be == "nccl":
        dist.barrier(group=group, device_ids=[torch.cuda.current_device()])
        return
    if monitored is None:
        monitored = os.environ.get("MADNN_MONITORED_BARRIER", "1") != "0"
    if monitored and be == "gloo":
        kw = {}
        if timeout_s is not None:
            kw["timeout"] = datetime.timedelta(seconds=timeout_s)
        dist.monitored_barrier(group=group, wait_all_ranks=True, **kw)
    else:
        dist.barrier(group=group)


def seed_all(seed: int, rank_offset: bool = False) -> None:
    """Same seed on every rank (as the reference example, sgd-...-cifar.lua:48)."""
    s = seed + (get_rank() if rank_offset else 0)
    random.seed(s)
    torch.manual_seed(s)
    try:
        import numpy as np

        np.random.seed(s % (2**32))
    except Exception:
        pass


AXES = ("dp", "pp", "cp", "tp")  # outermost -> innermost rank order


@dataclass(frozen=True)
class Mesh:
    """Logical device mesh over the world: data x pipeline x context x tensor parallel.

    ``cp`` (context / sequence parallel) is the extension axis SURVEY §5.7 asks for: no BASELINE
    config needs it, so it defaults to 1, but its process groups already exist, so ring attention
    or Ulysses can be added without changing this API.  Ranks are laid out tp innermost, then cp,
    pp and dp."""

    dp: int
    pp: int
    tp: int
    cp: int = 1

    @property
    def size(self) -> int:
        return self.dp * self.pp * self.cp * self.tp

    def _dims(self):
        return [getattr(self, a) for a in AXES]

    def coord(self, rank: int) -> dict:
        """rank -> {axis: index} for every axis."""
        out = {}
        for a, n in zip(reversed(AXES), reversed(self._dims())):
            out[a] = rank % n
            rank //= n
        return out

    def coords(self, rank: int):
        """rank -> (dp_idx, pp_idx, tp_idx) (the cp index is in :meth:`coord`)."""
        c = self.coord(rank)
        return c["dp"], c["pp"], c["tp"]

    def rank_of(self, dp_i: int, pp_i: int, tp_i: int, cp_i: int = 0) -> int:
        return ((dp_i * self.pp + pp_i) * self.cp + cp_i) * self.tp + tp_i

    def axis_groups(self, axis: str):
        """Every rank list that varies only along ``axis`` (one group per other-axes coordinate)."""
        if axis not in AXES:
            raise KeyError(f"unknown mesh axis {axis!r}; expected one of {AXES}")
        groups = {}
        for r in range(self.size):
            c = self.coord(r)
            key = tuple(c[a] for a in AXES if a != axis)
            groups.setdefault(key, []).append(r)
        return [groups[k] for k in sorted(groups)]


class ProcessGroups:
    """dp / pp / cp / tp sub-groups over the world (every rank creates every group
    in the same order, as torch.distributed requires).

    On one MI355X node all 8 GPUs are xGMI peers (7 links each), so no axis is
    placed for hop count; the DP all-reduce (same stage, different replicas)
    and the PP send/recv (adjacent stages) use disjoint links.
    An axis of size one gets a :class:`LocalGroup` (no communicator, no stream);
    an axis spanning the whole world is the world group (``None``).
    """

    _cache: dict = {}

    def __init__(self, mesh: Mesh):
        world = get_world_size()
        if mesh.size != world:
            raise ValueError(f"mesh {mesh} does not cover world size {world}")
        self.mesh = mesh
        self.rank = get_rank()
        c = mesh.coord(self.rank)
        self.dp_idx, self.pp_idx, self.cp_idx, self.tp_idx = c["dp"], c["pp"], c["cp"], c["tp"]
        for axis in AXES:
            setattr(self, f"{axis}_group", None)
            setattr(self, f"{axis}_ranks", next(g for g in mesh.axis_groups(axis) if self.rank in g))
        if not dist.is_initialized():
            return
        for axis in AXES:
            for ranks in mesh.axis_groups(axis):
                key = tuple(ranks)
                if key not in ProcessGroups._cache:
                    if len(ranks) == world:
                        ProcessGroups._cache[key] = None            # the world group itself
                    elif len(ranks) == 1:
                        ProcessGroups._cache[key] = LocalGroup(ranks[0])   # no communicator
                    else:
                        ProcessGroups._cache[key] = dist.new_group(list(ranks))
                if self.rank in ranks:
                    setattr(self, f"{axis}_group", ProcessGroups._cache[key])


def topology() -> dict:
    """Best-effort GPU link topology (rocm-smi); informational only."""
    info = {"gpus": torch.cuda.device_count() if torch.cuda.is_available() else 0}
    try:
        out = subprocess.run(["rocm-smi", "--showtopotype"], capture_output=True, text=True, timeout=20)
        info["xgmi"] = "XGMI" in out.stdout
        info["raw"] = out.stdout[-2000:]
    except Exception:
        info["xgmi"] = None
    return info
