"""Strategy-agnostic checkpoints (save / load / consolidate / resume).

The reference has no checkpointing at all: no torch.save of
models or optimizer state, and the trainer's sync counter lives only on the
object.  madnn's format::

    <dir>/madnn_meta.json              plan (strategy, dp/pp/tp, stage bounds,
                                       microbatches, sync mode/period/counter),
                                       step, world size, versions, shard list
    <dir>/model-<shard>.safetensors    fp32 master weights + buffers, keyed by the
                                       UN-WRAPPED single-device parameter names
    <dir>/optim-<shard>.pt             optimizer state per parameter name (plain
                                       tensors only: loads with weights_only=True)
    <dir>/state-<coords>.pt            per-rank resume state keyed by MESH coordinates
                                       (e.g. ``dp1-pp0-tp0``): RNG, data-sampler
                                       cursor, trainer epoch/position, the
                                       ``parallelize`` auto-sync counter

One shard per pipeline stage, written by that stage's DP-rank 0.  Because keys
are the original model's names, ``consolidate()`` merges the shards into one
state dict that loads into plain PyTorch, and ``load()`` restores into ANY
placement (different world size / strategy) by name — re-planning is free.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional

import torch
from torch import nn

from .. import runtime as rt

FORMAT = "madnn-ckpt-v1"


def _st():
    from safetensors.torch import load_file, save_file

    return save_file, load_file


def _named_state(engine) -> Dict[str, torch.Tensor]:
    """name -> fp32 FULL value of every parameter this rank holds, plus buffers.  Collective
    for tensor-parallel shards (gathered over their TP group, with or without a DP space)."""
    from ..parallel.dp import DataParallel
    from ..parallel.pp import PipelineEngine

    out = {}
    if isinstance(engine, PipelineEngine):
        space = engine.dp.space
        for name, p in engine.state_dict().items():
            out[name] = space.master_view(p).detach().float().cpu().contiguous() if id(p) in space.param_info \
                else p.detach().float().cpu()
        for name, b in engine.named_buffers():
            out[name] = b.detach().cpu().clone()
        return out
    module = engine.module if isinstance(engine, DataParallel) else engine
    space = engine.space if isinstance(engine, DataParallel) else None
    seen = {}
    for name, p in module.named_parameters(remove_duplicate=False):
        if id(p) in seen:  # tied weight: store once, record the alias
            out.setdefault("__aliases__", {})[name] = seen[id(p)]
            continue
        seen[id(p)] = name
        v = space.master_view(p) if space is not None and id(p) in space.param_info else p
        out[name] = _full_value(module, name, v.detach().float()).cpu().contiguous()
    for name, b in module.named_buffers():
        out[name] = b.detach().cpu().clone()
    return out


def _tp_owner(module, name):
    """(owner layer, attribute, shard dim) for a parameter sharded by tensor parallelism, else None."""
    from ..parallel.tp import ColumnParallelLinear, RowParallelLinear, _world

    owner_name, _, attr = name.rpartition(".")
    try:
        owner = module.get_submodule(owner_name) if owner_name else module
    except AttributeError:
        return None
    if isinstance(owner, RowParallelLinear) and attr == "weight" and _world(owner.group) > 1:
        return owner, attr, 1
    if isinstance(owner, ColumnParallelLinear) and _world(owner.group) > 1:
        return owner, attr, 0
    return None


def _full_value(module, name, t: torch.Tensor) -> torch.Tensor:
    """Gather a TP shard (any tensor shaped like the local parameter: value or optimizer state)
    to the full parameter shape; other tensors pass through."""
    own = _tp_owner(module, name)
    if own is None:
        return t
    owner, _attr, dim = own
    from .. import comm
    from ..parallel.tp import _world

    w = _world(owner.group)
    t = t.contiguous()
    buf = torch.empty((w * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    if dim == 0:
        comm.all_gather_into(buf, t, group=owner.group)
        return buf
    tt = t.t().contiguous()  # row-parallel weight [out, in/W]: gather the in-dim as rows
    buf = torch.empty((w * tt.shape[0], tt.shape[1]), dtype=t.dtype, device=t.device)
    comm.all_gather_into(buf, tt, group=owner.group)
    return buf.t().contiguous()


def _local_value(module, name, full: torch.Tensor, local_shape) -> torch.Tensor:
    """This rank's shard of a FULL tensor (inverse of :func:`_full_value`)."""
    own = _tp_owner(module, name)
    if own is None or tuple(full.shape) == tuple(local_shape):
        return full
    owner, _attr, dim = own
    from ..parallel.tp import _rank

    k = local_shape[dim]
    r = _rank(owner.group)
    return full.narrow(dim, r * k, k)


def _full_param(module, name, p):
    """Gather TP-sharded weights back to their full shape."""
    return _full_value(module, name, p.detach())


def _optim_state(engine, optimizer) -> Dict[str, Dict[str, torch.Tensor]]:
    """Per-parameter optimizer state under the parameters' names, TP shards gathered to the
    full shape (collective: every rank calls it with the same parameter order)."""
    from ..parallel.dp import DataParallel

    if optimizer is None:
        return {}
    sd = optimizer.state_dict()
    idx2p = {}
    k = 0
    for g in optimizer.param_groups:
        for p in g["params"]:
            idx2p[k] = p
            k += 1
    names = _param_names(engine)
    module = engine.module if isinstance(engine, DataParallel) else engine
    out = {}
    for i in sorted(sd["state"], key=int):
        st = sd["state"][i]
        p = idx2p.get(int(i))
        if p is None or id(p) not in names:
            continue
        name = names[id(p)]
        ent = {}
        for kk, v in st.items():
            if isinstance(v, torch.Tensor) and tuple(v.shape) == tuple(p.shape) and isinstance(module, nn.Module):
                v = _full_value(module, name, v.to(p.device))
            ent[kk] = v.detach().cpu() if isinstance(v, torch.Tensor) else torch.tensor(v)
        out[name] = ent
    return out


def _param_names(engine) -> Dict[int, str]:
    from ..parallel.dp import DataParallel
    from ..parallel.pp import PipelineEngine

    if isinstance(engine, PipelineEngine):
        return {id(p): n for n, p in engine.state_dict().items()}
    module = engine.module if isinstance(engine, DataParallel) else engine
    return {id(p): n for n, p in module.named_parameters()}


def _shard_id(engine) -> Optional[int]:
    """Which shard this rank writes (None = this rank writes nothing)."""
    from ..parallel.pp import PipelineEngine

    if isinstance(engine, PipelineEngine):
        return engine.stage if engine.groups.dp_idx == 0 else None
    return 0 if rt.get_rank() == 0 else None


def _coords(engine) -> dict:
    """This rank's mesh coordinates {"dp", "pp", "tp"} under ``engine``'s placement."""
    g = getattr(engine, "groups", None)
    if g is None and hasattr(engine, "module"):
        g = getattr(engine.module, "groups", None)
    if g is not None:
        return {"dp": g.dp_idx, "pp": g.pp_idx, "tp": g.tp_idx}
    return {"dp": rt.get_rank(), "pp": 0, "tp": 0}


def _coord_name(c: dict) -> str:
    return f"dp{c['dp']}-pp{c['pp']}-tp{c['tp']}"


def _periodic_sync(engine):
    from ..parallel.dp import DataParallel

    module = engine.module if isinstance(engine, DataParallel) else engine
    return getattr(module, "_madnn_sync", None) if isinstance(module, nn.Module) else None


def _resume_state(engine, sampler, trainer) -> dict:
    out = {"rng_cpu": torch.get_rng_state()}
    if torch.cuda.is_available():
        out["rng_cuda"] = torch.cuda.get_rng_state()
    ps = _periodic_sync(engine)
    if ps is not None:
        out["sync"] = {"counter": ps.counter, "period": ps.period, "backwards": ps.backwards, "syncs": ps.syncs}
    if sampler is not None:
        out["sampler"] = sampler.state_dict()
    if trainer is not None:
        out["trainer"] = trainer.state_dict()
    return out


def save(path: str, engine, optimizer=None, step: int = 0, extra: Optional[dict] = None, sampler=None,
         trainer=None) -> None:
    """Collective: every rank calls it; DP-rank 0 of every stage writes its shard, and every rank
    writes its resume state (RNG, ``sampler`` cursor, ``trainer`` position, the auto-sync
    counter of a ``parallelize``-d model) under its mesh coordinates."""
    save_file, _ = _st()
    os.makedirs(path, exist_ok=True)
    state = _named_state(engine)          # collective for TP gathers: all ranks
    aliases = state.pop("__aliases__", {})
    ostate = _optim_state(engine, optimizer)
    shard = _shard_id(engine)
    if shard is not None:
        save_file(state, os.path.join(path, f"model-{shard:05d}.safetensors"))
        flat = {}
        for name, st in ostate.items():
            for k, v in st.items():
                flat[f"{name}::{k}"] = v
        torch.save(flat, os.path.join(path, f"optim-{shard:05d}.pt"))
    coords = _coords(engine)
    torch.save(_resume_state(engine, sampler, trainer), os.path.join(path, f"state-{_coord_name(coords)}.pt"))
    rt.barrier()
    if rt.get_rank() == 0:
        meta = {"format": FORMAT, "time": time.time(), "step": int(step), "world": rt.get_world_size(),
                "torch": torch.__version__, "plan": _plan_meta(engine), "extra": extra or {},
                "aliases": aliases, "mesh": _mesh_meta(engine), "optim_groups": _group_hparams(optimizer),
                "shards": sorted(f for f in os.listdir(path) if f.startswith("model-"))}
        with open(os.path.join(path, "madnn_meta.json"), "w") as f:
            json.dump(meta, f, indent=2)
    rt.barrier()


def _group_hparams(optimizer) -> list:
    """JSON-able hyper-parameters of every optimizer param group (lr, momentum, betas, ...)."""
    if optimizer is None:
        return []
    out = []
    for g in optimizer.param_groups:
        d = {}
        for k, v in g.items():
            if k == "params":
                continue
            if isinstance(v, (int, float, bool, str)) or v is None:
                d[k] = v
            elif isinstance(v, (tuple, list)) and all(isinstance(x, (int, float)) for x in v):
                d[k] = list(v)
        out.append(d)
    return out


def _mesh_meta(engine) -> dict:
    g = getattr(engine, "groups", None)
    if g is None and hasattr(engine, "module"):
        g = getattr(engine.module, "groups", None)
    if g is not None:
        m = g.mesh
        return {"dp": m.dp, "pp": m.pp, "tp": m.tp}
    return {"dp": rt.get_world_size(), "pp": 1, "tp": 1}


def _plan_meta(engine) -> dict:
    from ..parallel.dp import DataParallel
    from ..parallel.pp import PipelineEngine

    if isinstance(engine, PipelineEngine):
        p = engine.plan
        return {"strategy": p.strategy, "dp": p.dp, "pp": p.pp, "bounds": p.bounds, "microbatches": p.microbatches,
                "schedule": engine.schedule}
    if isinstance(engine, DataParallel):
        return {"strategy": "dp", "dp": engine.world, "pp": 1, "sync": engine.sync, "sync_every": engine.sync_every,
                "sync_samples": engine.sync_samples, "sync_calibration": engine.sync_calibration,
                "steps": engine._steps, "samples": engine._samples, "per_step": engine._per_step,
                "period_origin": engine._period_origin}
    return {"strategy": "none"}


def consolidate(path: str) -> Dict[str, torch.Tensor]:
    """Merge every model shard into one plain state dict (loads into the un-wrapped model)."""
    _, load_file = _st()
    out = {}
    for f in sorted(os.listdir(path)):
        if f.startswith("model-") and f.endswith(".safetensors"):
            out.update(load_file(os.path.join(path, f)))
    meta_f = os.path.join(path, "madnn_meta.json")
    if os.path.exists(meta_f):
        with open(meta_f) as fh:
            for alias, canon in json.load(fh).get("aliases", {}).items():
                if alias not in out and canon in out:
                    out[alias] = out[canon]
    return out


def _optim_all(path: str) -> Dict[str, Dict[str, torch.Tensor]]:
    out: Dict[str, Dict[str, torch.Tensor]] = {}
    for f in sorted(os.listdir(path)):
        if f.startswith("optim-") and f.endswith(".pt"):
            flat = torch.load(os.path.join(path, f), map_location="cpu", weights_only=True)
            for key, v in flat.items():
                name, _, k = key.partition("::")
                out.setdefault(name, {})[k] = v
    return out


def load(path: str, engine, optimizer=None, strict: bool = True, sampler=None, trainer=None) -> dict:
    """Restore weights (and optimizer state) into any placement, by parameter name; plus this
    rank's resume state (RNG, sampler cursor, trainer position, auto-sync counter).  The resume
    state is looked up by mesh coordinates; at a different placement a rank takes the state of
    the saved coordinates it maps onto (dp index modulo the saved dp size), which keeps the
    data position but cannot reproduce per-rank random streams bit for bit."""
    from ..parallel.dp import DataParallel
    from ..parallel.pp import PipelineEngine

    with open(os.path.join(path, "madnn_meta.json")) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT:
        raise ValueError(f"not a madnn checkpoint: {path}")
    full = consolidate(path)
    names = _param_names(engine)
    space = None
    if isinstance(engine, PipelineEngine):
        space = engine.dp.space
        params = {n: p for n, p in engine.state_dict().items()}
        module = engine.module
    elif isinstance(engine, DataParallel):
        space = engine.space
        module = engine.module
        params = dict(module.named_parameters())
    else:
        module = engine
        params = dict(module.named_parameters())
    missing = [n for n in params if n not in full]
    if strict and missing:
        raise KeyError(f"checkpoint misses parameters: {missing[:5]}")
    with torch.no_grad():
        for n, p in params.items():
            if n not in full:
                continue
            v = _local_value(module, n, full[n], tuple(p.shape))
            if space is not None and id(p) in space.param_info:
                space.master_view(p).copy_(v.to(space.master_view(p).device))
            else:
                p.copy_(v.to(p.device))
        if space is not None:
            space.sync_model_from_master()
        bufs = dict(engine.named_buffers()) if isinstance(engine, PipelineEngine) else dict(module.named_buffers())
        for n, b in bufs.items():
            if n in full:
                b.copy_(full[n].to(b.device))
    if optimizer is not None:
        ost = _optim_all(path)
        sd = optimizer.state_dict()
        k = 0
        new_state = {}
        for g in optimizer.param_groups:
            for p in g["params"]:
                n = names.get(id(p))
                if n in ost:
                    new_state[k] = {kk: (_local_value(module, n, v, tuple(p.shape))
                                         if isinstance(v, torch.Tensor) and v.dim() == p.dim() and v.dim() > 0 else v)
                                    for kk, v in ost[n].items()}
                k += 1
        sd["state"] = new_state
        saved = meta.get("optim_groups") or []
        if len(saved) == len(sd["param_groups"]):
            for g, h in zip(sd["param_groups"], saved):
                for k, v in h.items():
                    g[k] = tuple(v) if isinstance(g.get(k), tuple) else v
        optimizer.load_state_dict(sd)
    if isinstance(engine, DataParallel):
        pm = meta.get("plan", {})
        engine._steps = int(pm.get("steps", engine._steps))
        # the sync="params" period resumes where it was: the sample counter, the agreed samples
        # per step, and (sync_every="auto") the measured K instead of a fresh calibration
        engine._samples = int(pm.get("samples") or 0)
        engine._per_step = pm.get("per_step")
        engine._period_origin = int(pm.get("period_origin") or 0)
        cal = pm.get("sync_calibration")
        if engine.sync_every == "auto" and cal and cal.get("K"):
            engine.sync_every = int(cal["K"])
            engine.sync_calibration = dict(cal, resumed=True)
    st = _load_resume_state(path, engine, meta)
    if st is not None:
        torch.set_rng_state(st["rng_cpu"])
        if "rng_cuda" in st and torch.cuda.is_available():
            torch.cuda.set_rng_state(st["rng_cuda"])
        ps = _periodic_sync(engine)
        if ps is not None and "sync" in st:
            ps.counter = int(st["sync"]["counter"])
            ps.backwards = int(st["sync"]["backwards"])
            ps.syncs = int(st["sync"]["syncs"])
        if sampler is not None and "sampler" in st:
            sampler.load_state_dict(st["sampler"])
        if trainer is not None and "trainer" in st:
            trainer.load_state_dict(st["trainer"])
    return meta


def _load_resume_state(path: str, engine, meta: dict) -> Optional[dict]:
    c = _coords(engine)
    f = os.path.join(path, f"state-{_coord_name(c)}.pt")
    mapped = None
    if not os.path.exists(f):
        saved = meta.get("mesh") or {"dp": meta.get("world", 1), "pp": 1, "tp": 1}
        mapped = {"dp": c["dp"] % max(int(saved["dp"]), 1), "pp": min(c["pp"], int(saved["pp"]) - 1),
                  "tp": c["tp"] % max(int(saved["tp"]), 1)}
        f = os.path.join(path, f"state-{_coord_name(mapped)}.pt")
    if not os.path.exists(f):
        legacy = os.path.join(path, f"rng-rank{rt.get_rank()}.pt")   # round-2 checkpoints
        if not os.path.exists(legacy):
            return None
        rng = torch.load(legacy, weights_only=True)
        return {"rng_cpu": rng["cpu"], **({"rng_cuda": rng["cuda"]} if "cuda" in rng else {})}
    st = torch.load(f, weights_only=True)
    if mapped is not None and (mapped["dp"], mapped["pp"]) != (c["dp"], c["pp"]):
        # a rank with no saved state of its own (resumed on a larger mesh) borrows another
        # coordinate's state: fold its dp / pp coordinates into the RNG streams, or it would draw
        # the same dropout masks as the replica it borrowed from.  The tp coordinate is NOT folded:
        # a tensor-parallel group's ranks must keep one shared stream (dropout on replicated
        # activations), and they borrow from one saved TP group, whose states are equal
        fold = {"dp": c["dp"], "pp": c["pp"]}
        st["rng_cpu"] = _fold_rng(st["rng_cpu"], fold)
        if "rng_cuda" in st:
            st["rng_cuda"] = _fold_rng(st["rng_cuda"], fold)
    return st


def _fold_rng(state: torch.Tensor, coords: dict) -> torch.Tensor:
    """A new generator state derived from ``state`` and the mesh coordinates (deterministic)."""
    import hashlib

    h = hashlib.sha256(state.numpy().tobytes() + repr(sorted(coords.items())).encode()).digest()
    g = torch.Generator()
    g.manual_seed(int.from_bytes(h[:8], "little") & ((1 << 63) - 1))
    if state.numel() == g.get_state().numel():
        return g.get_state()
    # a device generator state (philox seed + offset): reseed its seed field
    out = state.clone()
    out[:8] = torch.tensor(list(h[:8]), dtype=torch.uint8)
    return out
