"""Auto-partitioner: trace -> cost -> place (DP, PP or DP x PP) for one node.

North-star requirement: walk an arbitrary ``nn.Module``,
cost each layer, and place it across the GPUs of one node as data- or
pipeline-parallel stages sized for 288 GB of HBM3E per GPU.  The reference's
closest analog is the sync-period heuristic (datamodule.lua:68-78) and the
dead ``comm_speed`` probe (datamodule.lua:280-303).

Step-time model for ``W = dp x pp`` GPUs, global batch B, M microbatches:

* DP   (pp = 1): compute(B/dp) + exposed all-reduce, where the bucketed
  all-reduce overlaps backward so only the last bucket (and whatever exceeds
  the backward time) is exposed;
* PP   (dp = 1): (M + pp - 1)/M x max_stage(B) + per-microbatch P2P of the
  boundary activations and gradients;
* DPxPP: the PP expression with B/dp per replica, plus the stage-local
  all-reduce over dp (on links disjoint from the PP hops).

Memory per GPU: parameter/optimizer bytes of its stage (madnn layout, 16-20
B/param) + saved activations (1F1B keeps ``pp - s`` microbatches in flight on
stage s; with activation checkpointing only boundary tensors + one layer).
A candidate that does not fit ``hbm_gb x mem_headroom`` first tries
checkpointing, then is dropped.  Stage boundaries come from the C++
min-max-bottleneck partitioner (``madnn_partition``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import torch
from torch import nn

from ..config import Config, torch_dtype
from ..ops import native_runtime
from .cost import LayerCost, divisors, estimate, stage_estimate
from .hw import Machine, load
from .trace import Spine, find_block_list, trace


@dataclass
class Plan:
    strategy: str                      # dp | pp | dp_pp
    dp: int
    pp: int
    bounds: List[int]                  # stage boundaries over spine layers (len pp+1)
    microbatches: int
    checkpoint: List[bool]             # per spine layer
    est_step_s: float
    est_mem_gb: List[float]            # per stage, per GPU
    spine: Optional[Spine] = None
    costs: Optional[List[LayerCost]] = None
    candidates: list = field(default_factory=list)
    global_batch: int = 0

    def describe(self) -> str:
        ck = sum(self.checkpoint)
        return (f"{self.strategy} dp={self.dp} pp={self.pp} stages={self.bounds} microbatches={self.microbatches} "
                f"ckpt_layers={ck}/{len(self.checkpoint)} est_step={self.est_step_s * 1e3:.1f}ms "
                f"mem/GPU={max(self.est_mem_gb):.1f}GB")

    def table(self) -> str:
        rows = ["| strategy | dp | pp | M | ckpt | est step (ms) | max mem/GPU (GB) | fits |", "|---|---|---|---|---|---|---|---|"]
        for c in self.candidates:
            rows.append(f"| {c['strategy']} | {c['dp']} | {c['pp']} | {c['M']} | {c['ckpt']} | "
                        f"{c['step_s'] * 1e3:.2f} | {c['mem_gb']:.1f} | {c['fits']} |")
        return "\n".join(rows)


def infer_example_input(model: nn.Module, batch: int = 1) -> torch.Tensor:
    """A representative input when the caller gives none (zoo configs, first layer shapes)."""
    cfg = getattr(model, "config", None)
    if cfg is not None:
        seq = getattr(cfg, "n_positions", None) or getattr(cfg, "max_position", None) or 512
        seq = min(seq, 2048)
        return torch.zeros(batch, seq, dtype=torch.long)
    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            return torch.zeros(batch, m.in_channels, 224, 224)
        if isinstance(m, nn.Linear):
            return torch.zeros(batch, m.in_features)
        if isinstance(m, nn.Embedding):
            return torch.zeros(batch, 512, dtype=torch.long)
    raise ValueError("cannot infer an example input; pass example_input=")


def _opt_kind(optimizer) -> str:
    if optimizer is None:
        return "adam"
    name = type(optimizer).__name__.lower()
    return "adam" if "adam" in name else "sgd"


def plan_model(model: nn.Module, cfg: Config, world: int, example_input: Optional[torch.Tensor] = None,
               optimizer=None, global_batch: Optional[int] = None, machine: Optional[Machine] = None) -> Plan:
    hw = machine or load()
    spine = trace(model)
    if example_input is None:
        example_input = infer_example_input(model)
    dtype = torch_dtype(cfg.dtype)
    costs = estimate(spine, example_input, dtype=dtype, machine=hw)
    B = global_batch or cfg.extra.get("global_batch") or max(example_input.shape[0], 1) * world
    opt = _opt_kind(optimizer)
    cap = hw.hbm_gb * cfg.mem_headroom * 1e9
    L = len(spine)
    forced = cfg.strategy
    cands = []
    for pp in divisors(world):
        if pp > L:
            continue
        dp = world // pp
        if not _allowed(forced, pp, dp, world, cfg.pp_stages):
            continue
        for ckpt_mode in ([False, True] if cfg.checkpointing == "auto" else [cfg.checkpointing == "all"]):
            c = _candidate(costs, pp, dp, B, cfg, hw, opt, cap, ckpt_mode)
            if c is not None:
                cands.append(c)
    if not cands:
        raise RuntimeError(f"madnn planner: no feasible placement for world={world}, strategy={forced}")
    feasible = [c for c in cands if c["fits"]] or cands
    best = min(feasible, key=lambda c: (c["step_s"], c["pp"], c["ckpt"]))
    strategy = "dp" if best["pp"] == 1 else ("pp" if best["dp"] == 1 else "dp_pp")
    ck = [best["ckpt"] and _ckpt_eligible(spine, i) for i in range(L)]
    return Plan(strategy, best["dp"], best["pp"], best["bounds"], best["M"], ck, best["step_s"], best["mem_list"],
                spine, costs, cands, B)


def _allowed(forced: str, pp: int, dp: int, world: int, pp_stages) -> bool:
    if forced == "dp":
        return pp == 1
    if forced == "pp":
        return pp == (pp_stages or world) and pp > 1 or world == 1
    if forced == "dp_pp":
        if pp_stages:
            return pp == pp_stages
        return 1 < pp < world or world == 1
    return True


def _ckpt_eligible(spine: Spine, i: int) -> bool:
    # checkpoint the repeated blocks, not the embedding/head ends
    return 0 < i < len(spine) - 1 or len(spine) == 1


def _candidate(costs, pp, dp, B, cfg, hw: Machine, opt, cap, ckpt):
    L = len(costs)
    per_replica = max(B // dp, 1)
    M = 1 if pp == 1 else (cfg.microbatches or min(max(4 * pp, pp), per_replica))
    M = max(1, min(M, per_replica))
    mb = per_replica / M
    times = [c.time_s * (1.0 + (1.0 / 3.0 if ckpt else 0.0)) for c in costs]
    mems = [stage_estimate(costs, i, i + 1, opt, ckpt).param_bytes + stage_estimate(costs, i, i + 1, opt, ckpt)
            .act_bytes_per_sample * mb * (pp if pp > 1 else 1) for i in range(L)]
    try:
        bounds, _ = native_runtime.partition(times, pp, mems, cap if cap > 0 else 0.0)
    except ValueError:
        bounds, _ = native_runtime.partition(times, pp)
    stage_t, mem_list = [], []
    for s in range(pp):
        lo, hi = bounds[s], bounds[s + 1]
        est = stage_estimate(costs, lo, hi, opt, ckpt)
        stage_t.append(est.time_per_sample_s * mb)
        inflight = (pp - s) if cfg.schedule == "1f1b" else M
        inflight = min(inflight, M)
        act = est.act_bytes_per_sample * mb * inflight
        mem_list.append((est.param_bytes + act) / 1e9)
    bottleneck = max(stage_t)
    if pp == 1:
        compute = bottleneck
        grad_bytes = sum(c.params for c in costs) * 4.0  # fp32 reduce buffers
        ar = hw.allreduce_s(grad_bytes, dp)
        exposed = max(ar - 0.8 * compute * (2.0 / 3.0), ar * 0.1)
        step = compute + exposed
    else:
        p2p = max(costs[bounds[s + 1] - 1].out_bytes * mb for s in range(pp - 1))
        step = (M + pp - 1) * bottleneck + 2 * (M + pp - 1) * hw.p2p_s(p2p)
        if dp > 1:
            stage_params = max(stage_estimate(costs, bounds[s], bounds[s + 1], opt).params for s in range(pp))
            step += 0.3 * hw.allreduce_s(stage_params * 4.0, dp)
    fits = max(mem_list) * 1e9 <= cap
    return {"strategy": "dp" if pp == 1 else ("pp" if dp == 1 else "dp_pp"), "dp": dp, "pp": pp, "M": M,
            "ckpt": ckpt, "bounds": bounds, "step_s": step, "mem_gb": max(mem_list), "mem_list": mem_list,
            "fits": fits}


__all__ = ["Plan", "plan_model", "trace", "estimate", "infer_example_input", "find_block_list"]
