"""Auto-partitioner: trace -> cost -> place (DP, PP, DP x PP or DP x TP) for one node.

North-star requirement: walk an arbitrary ``nn.Module``,
cost each layer, and place it across the GPUs of one node as data- or
pipeline-parallel stages sized for 288 GB of HBM3E per GPU.  The reference's
closest analog is the sync-period heuristic (datamodule.lua:68-78) and the
dead ``comm_speed`` probe (datamodule.lua:280-303).

Costs: per-layer analytic FLOPs/bytes on the meta device (``cost.estimate``),
replaced by HIP-event measurements of every distinct layer when a GPU is
present (``cost.measure_layers``).  Machine numbers (xGMI all-reduce / P2P
bandwidth, HBM, GEMM rate) come from the calibrated hardware profile
(``madnn.planner.calibrate``) when one exists, else the datasheet defaults.

Step-time model for ``W = dp x pp x tp`` GPUs, global batch B, M microbatches:

* DP: compute(B/dp) + the part of the bucketed all-reduce that the backward
  does not hide -- a bucket-by-bucket timeline: buckets fill in backward
  order, each is reduced when its last gradient lands, one after another on
  the comm stream; exposed = reductions still running after backward ends;
* PP (GPipe / 1F1B / interleaved with V chunks per rank): the makespan of the
  engine's own transport (``parallel.pp.simulate_transport``: the boundary-batched
  issue plan with the node's measured P2P time), i.e. the schedule's bubble plus
  whatever transfers the schedule leaves on the critical path; with dp > 1 the
  stage-local all-reduce overlaps only the last microbatch's backward (same
  timeline);
* TP (row-parallel large Linears, ``strategy="tp"``): the sharded GEMM share of
  compute divided by T, plus the per-layer activation all-reduce and
  input-gradient all-gather on the critical path.

Memory per GPU: parameter/optimizer bytes of its layers (madnn layout)
+ saved activations of the microbatches in flight (simulated per schedule;
with activation checkpointing only boundary tensors + one layer).  A candidate
that does not fit ``hbm_gb x mem_headroom`` is dropped unless nothing fits.
Stage boundaries come from the C++ min-max-bottleneck partitioner
(``madnn_partition``).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
from torch import nn

from ..config import Config, torch_dtype
from ..ops import native_runtime
from ..utils.logging import get_logger
from .cost import (LayerCost, MeasurementFailed, divisors, estimate, measure_chain, measure_layers, param_state_bytes,
                   stage_estimate)
from .hw import Machine, load
from .trace import Spine, find_block_list, trace


@dataclass
class Plan:
    strategy: str                      # dp | pp | dp_pp | tp
    dp: int
    pp: int
    bounds: List[int]                  # chunk boundaries over spine layers (len pp*virtual+1)
    microbatches: int
    checkpoint: List[bool]             # per spine layer
    est_step_s: float
    est_mem_gb: List[float]            # per pipeline rank, per GPU
    spine: Optional[Spine] = None
    costs: Optional[List[LayerCost]] = None
    candidates: list = field(default_factory=list)
    global_batch: int = 0
    schedule: str = "1f1b"
    virtual: int = 1
    tp: int = 1
    measured: bool = False

    def describe(self) -> str:
        ck = sum(self.checkpoint)
        sched = f" schedule={self.schedule}" + (f"x{self.virtual}" if self.virtual > 1 else "") if self.pp > 1 else ""
        return (f"{self.strategy} dp={self.dp} pp={self.pp} tp={self.tp}{sched} stages={self.bounds} "
                f"microbatches={self.microbatches} ckpt_layers={ck}/{len(self.checkpoint)} "
                f"est_step={self.est_step_s * 1e3:.1f}ms mem/GPU={max(self.est_mem_gb):.1f}GB "
                f"costs={'measured' if self.measured else 'analytic'}")

    def table(self) -> str:
        rows = ["| strategy | dp | pp | tp | sched | M | ckpt | compute (ms) | exposed comm (ms) | bubble | "
                "est step (ms) | max mem/GPU (GB) | fits |",
                "|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
        for c in sorted(self.candidates, key=lambda c: c["step_s"]):
            sched = c.get("schedule", "-") + (f" V={c['V']}" if c.get("V", 1) > 1 else "")
            rows.append(f"| {c['strategy']} | {c['dp']} | {c['pp']} | {c.get('tp', 1)} | {sched} | "
                        f"{c['M']} | {c['ckpt']} | {c.get('compute_s', 0) * 1e3:.2f} | "
                        f"{c.get('comm_s', 0) * 1e3:.2f} | {c.get('bubble', 0):.3f} | {c['step_s'] * 1e3:.2f} | "
                        f"{c['mem_gb']:.1f} | {c['fits']} |")
        return "\n".join(rows)


def infer_example_input(model: nn.Module, batch: int = 1) -> torch.Tensor:
    """A representative input when the caller gives none (zoo configs, first layer shapes)."""
    cfg = getattr(model, "config", None)
    if cfg is not None:
        seq = getattr(cfg, "n_positions", None) or getattr(cfg, "max_position", None) or \
            getattr(cfg, "max_position_embeddings", None) or 512
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


def _reduce_bytes(cfg: Config) -> int:
    return 4 if cfg.reduce_dtype in ("float32", "fp32") else 2


def _bucket_bytes(cfg: Config, costs, rb: int) -> float:
    from ..config import auto_bucket_mb

    return (cfg.bucket_mb or auto_bucket_mb(sum(c.params for c in costs) * rb)) * 2**20


def _want_measure(cfg: Config) -> bool:
    v = cfg.extra.get("measure", os.environ.get("MADNN_PLAN_MEASURE", "auto"))
    if isinstance(v, str):
        v = v.lower()
        if v == "auto":
            return torch.cuda.is_available()
        return v in ("1", "true", "yes", "on")
    return bool(v)


def plan_model(model: nn.Module, cfg: Config, world: int, example_input: Optional[torch.Tensor] = None,
               optimizer=None, global_batch: Optional[int] = None, machine: Optional[Machine] = None,
               costs: Optional[List[LayerCost]] = None) -> Plan:
    """Trace, cost (measured on the GPU when available) and choose the placement with the
    lowest modelled step time that fits in HBM.  ``global_batch``: samples per optimizer step
    over the whole job (default ``cfg.extra['global_batch']``, else the example input's
    batch per GPU x ``world``)."""
    import time

    t_start = time.perf_counter()
    hw = machine or _job_machine()
    spine = trace(model)
    explicit_input = example_input is not None
    if example_input is None:
        example_input = infer_example_input(model)
    dtype = torch_dtype(cfg.dtype)
    measured = False
    B = global_batch or cfg.extra.get("global_batch")
    if not B:
        if not explicit_input:
            get_logger().warning("madnn planner: no example_input / global_batch given; assuming %d sample(s) per "
                                 "GPU for microbatch and activation sizing", example_input.shape[0])
        B = max(example_input.shape[0], 1) * world
    calib = None
    if costs is None:
        costs = estimate(spine, example_input, dtype=dtype, machine=hw)
        import torch.distributed as dist

        multi = dist.is_initialized() and dist.get_world_size() > 1
        if _want_measure(cfg):
            per_gpu = max(int(B) // max(world, 1), 1) if (explicit_input or global_batch
                                                          or cfg.extra.get("global_batch")) else None
            mb = int(cfg.extra.get("measure_batch", 0)) or _default_measure_batch(example_input, per_gpu)
            try:
                # every rank times its share of the distinct layers; the ranks agree on success
                # before the results are all-gathered (MeasurementFailed on every rank otherwise)
                costs = measure_layers(spine, example_input, costs, batch=mb, dtype=dtype,
                                       device=None if torch.cuda.is_available() else torch.device("cpu"))
            except MeasurementFailed as e:
                get_logger().warning("madnn planner: layer measurement failed (%s); using analytic costs", e)
                costs = estimate(spine, example_input, dtype=dtype, machine=hw)
            else:
                calib = _calibrate_chain(spine, example_input, costs, mb, dtype, cfg, hw)
        if multi:
            # every rank must choose the SAME placement: rank 0's (measured) costs are the plan input
            obj = [[(c.fwd_s, c.bwd_s, c.fixed_s, c.measured, c.act_bytes) for c in costs], calib]
            dist.broadcast_object_list(obj, src=0)
            for c, (f, b, fx, m, ab) in zip(costs, obj[0]):
                c.fwd_s, c.bwd_s, c.fixed_s, c.measured, c.act_bytes = f, b, fx, m, ab
            calib = obj[1]
    measured = all(c.measured for c in costs)
    comm_probe = _probe_comm(cfg, world)
    if comm_probe:
        from ..comm import probe as _probe

        hw = _probe.apply(hw, comm_probe)
    opt = _opt_kind(optimizer)
    cap = hw.hbm_gb * cfg.mem_headroom * 1e9
    L = len(spine)
    forced = cfg.strategy
    elig = [_ckpt_eligible(spine, i) for i in range(L)]
    cands = []
    for pp in divisors(world):
        if pp > L:
            continue
        dp = world // pp
        if not _allowed(forced, pp, dp, world, cfg.pp_stages):
            continue
        # checkpointing="auto": no recompute, every block, and the per-block choice (the fewest
        # blocks per rank whose recompute makes it fit, _candidate) are all priced
        modes = [False, True, "auto"] if cfg.checkpointing == "auto" else [cfg.checkpointing == "all"]
        for ckpt_mode in modes:
            for schedule, V, M in pp_variants(pp, max(B // dp, 1), L, cfg):
                c = _candidate(costs, pp, dp, B, cfg, hw, opt, cap, ckpt_mode, schedule, V, M, elig=elig)
                if c is not None:
                    cands.append(c)
    if (forced == "tp" or forced == "auto" and not cfg.pp_stages) and world > 1:
        for tp in divisors(world):
            if tp == 1 or (forced == "tp" and cfg.tp_size > 1 and tp != cfg.tp_size):
                continue
            c = _tp_candidate(spine, costs, world // tp, tp, B, cfg, hw, opt, cap, tuple(example_input.shape[1:]),
                              example_input.dtype)
            if c is not None:
                cands.append(c)
    if not cands:
        raise RuntimeError(f"madnn planner: no feasible placement for world={world}, strategy={forced}")
    feasible = [c for c in cands if c["fits"]] or cands
    best = min(feasible, key=lambda c: (c["step_s"], c["pp"], c.get("tp", 1), c["ckpt"]))
    ck = list(best.get("ck") or [False] * L)
    plan = Plan(best["strategy"], best["dp"], best["pp"], best["bounds"], best["M"], ck, best["step_s"],
                best["mem_list"], spine, costs, cands, B, schedule=best.get("schedule", "1f1b"),
                virtual=best.get("V", 1), tp=best.get("tp", 1), measured=measured)
    plan.calibration = calib
    plan.p2p_lag = best.get("lag", 0.0)   # the pipeline engine's second issue plan (pp.issue_plan)
    plan.comm_probe = comm_probe
    plan.machine = hw
    plan.plan_s = time.perf_counter() - t_start
    log = get_logger()
    log.info("madnn plan: %s", plan.describe())
    log.info("madnn plan candidates (world=%d, global batch %d):\n%s", world, B, plan.table())
    return plan


def _job_machine() -> Machine:
    """The machine profile of THIS job: the MI355X profile (``hw.load``), or the host-CPU one when
    the job really runs on CPU tensors over gloo."""
    import torch.distributed as dist

    from .. import runtime as rt
    from .hw import host_cpu

    if dist.is_initialized() and dist.get_backend() == "gloo" and rt.device().type == "cpu":
        return host_cpu()
    return load()


def _probe_comm(cfg: Config, world: int) -> Optional[dict]:
    """Measured all-reduce / P2P numbers of THIS job's world group (``comm.probe``), when the
    job really runs ``world`` > 1 ranks on RCCL or gloo; None otherwise (single GPU, a fake
    process group planning a hypothetical node, or ``MADNN_PLAN_COMM=0``)."""
    import torch.distributed as dist

    from ..comm import probe as _probe

    if not (dist.is_initialized() and world > 1 and dist.get_world_size() == world
            and dist.get_backend() in ("nccl", "gloo") and _probe.wanted(cfg)):
        return None
    res = _probe.measure()
    if res:
        get_logger().info("madnn planner: measured comm world=%d: all-reduce %.1f GB/s busbw, %.0f us small, "
                          "P2P %.1f GB/s", world, res["allreduce_busbw_gbps"], res["allreduce_small_us"],
                          res["p2p_gbps"])
    return res or None


def _default_measure_batch(example_input: torch.Tensor, per_gpu: Optional[int] = None) -> int:
    """Per-layer timing batch.  Per-sample costs fall steeply with the batch (a ResNet-50 layer at
    32 images runs at ~1/6 of its batch-2048 efficiency), so when the job's per-GPU batch is known
    the layers are timed at that batch, capped at 2048 images / 64k tokens / 1024 rows to bound the
    probe's memory and time; otherwise at a small default (~4k tokens, 32 images, 64 rows)."""
    per = int(torch.tensor(example_input.shape[1:]).prod()) if example_input.dim() > 1 else 1
    if example_input.dtype in (torch.long, torch.int32):  # token ids
        base, cap = max(1, min(16, 4096 // max(per, 1))), max(1, 65536 // max(per, 1))
    elif example_input.dim() == 4:
        base, cap = 32, 2048
    else:
        base, cap = 64, 1024
    return max(1, min(int(per_gpu), cap)) if per_gpu else base


def _allowed(forced: str, pp: int, dp: int, world: int, pp_stages) -> bool:
    if forced == "auto" and pp_stages:   # automatic everything except the pinned stage count
        return pp == pp_stages
    if forced == "dp":
        return pp == 1
    if forced == "tp":
        return False
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


def dp_exposed_s(bwd_times: List[float], grad_bytes: List[float], dp: int, hw: Machine, bucket_bytes: float) -> float:
    """Communication left exposed after backward by the overlapped bucketed all-reduce.

    ``bwd_times``/``grad_bytes`` per layer in FORWARD order (seconds for this rank's batch,
    bytes of its gradients in the reduce dtype).  Backward visits layers in reverse; a
    bucket (filled in that order up to ``bucket_bytes``) becomes ready when the backward of
    its last layer ends, and buckets are reduced one after another on the comm stream."""
    if dp <= 1:
        return 0.0
    t = 0.0
    ready = []
    cur = 0.0
    for bt, gb in zip(reversed(bwd_times), reversed(grad_bytes)):
        t += bt
        cur += gb
        if cur >= bucket_bytes:
            ready.append((t, cur))
            cur = 0.0
    if cur > 0:
        ready.append((t, cur))
    end = 0.0
    for rt_, nb in ready:
        end = max(end, rt_) + hw.allreduce_s(nb, dp)
    return max(0.0, end - t)


def _chunk_ranks(pp: int, V: int):
    return [[c * pp + r for c in range(V)] for r in range(pp)]


def pp_variants(pp: int, per_replica: int, L: int, cfg: Config):
    """The pipeline schedules the planner prices for ``pp`` stages: GPipe, 1F1B and interleaved
    1F1B with V in {2, 4} model chunks per rank, each at every microbatch count M in
    {pp, 2pp, 4pp, 8pp, 16pp} that divides the replica's batch (interleaving also needs
    M % pp == 0 and pp*V <= layers).  An explicit ``cfg.schedule`` / ``cfg.microbatches`` /
    ``cfg.virtual_stages`` narrows the search to it.  ``pp == 1`` yields the single DP variant."""
    if pp == 1:
        yield "none", 1, 1
        return
    scheds = ["gpipe", "1f1b", "interleaved"] if cfg.schedule in (None, "auto") else [cfg.schedule]
    if cfg.microbatches:
        ms = [max(1, min(int(cfg.microbatches), per_replica))]
    else:
        ms = sorted({m for m in (pp, 2 * pp, 4 * pp, 8 * pp, 16 * pp) if m <= per_replica and per_replica % m == 0})
        if not ms:  # a tiny batch: as many microbatches as it splits into evenly
            ms = [max(d for d in divisors(per_replica) if d <= pp)]
    for sched in scheds:
        if sched == "interleaved":
            vs = [int(cfg.virtual_stages)] if cfg.virtual_stages else [2, 4]
            for V in vs:
                if V < 2 or pp * V > L:
                    continue
                for M in ms:
                    if M % pp == 0:
                        yield "interleaved", V, M
        else:
            for M in ms:
                yield sched, 1, M


def optimizer_s(params: float, opt: str, hw: Machine) -> float:
    """The fused optimizer pass over ``params`` parameters: an HBM stream of the fp32 master,
    the reduced gradient, the state and the bf16 compute copy (Adam ~28 B, SGD ~20 B per
    parameter) at the profile's streaming bandwidth."""
    per = 28.0 if opt == "adam" else 20.0
    return params * per / (hw.hbm_tbps * 1e12)


def _agreed_min(x: float) -> float:
    """MIN of ``x`` over the job's ranks (``x`` itself without a multi-rank process group)."""
    import torch.distributed as dist

    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(x)
    v = torch.tensor([float(x)], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(v, op=dist.ReduceOp.MIN)
    return float(v)


def _calibrate_chain(spine, example_input, costs, batch, dtype, cfg: Config, hw: Machine):
    """Scale the per-layer costs so their sum matches ONE timing of the whole spine at the
    measurement batch (isolated layer timings miss what neighbouring layers do to each other).
    The same forward also measures the saved-activation bytes and rescales every layer's
    ``act_bytes`` to them.  When weights + gradients + the (estimated) activations of ``batch``
    samples would not fit 3/4 of the free HBM, the chain runs at batch / 2^k that does: the memory
    ratio is taken there, the timing ratio is not (a smaller batch has other neighbour effects) --
    the activation estimate over-counts most exactly when it is large, and that is when the
    planner most needs it corrected (GPT-2 medium at 128 sequences: 328 GB estimated, 129 GB
    measured).  Skipped when the weights alone take more than a quarter of HBM.  Returns
    ``{"ratio", "chain_s", "layers_s", "batch", "act_ratio", "saved_bytes", "chain_batch"}`` or None."""
    if not cfg.extra.get("calibrate_chain", True):
        return None
    nparams = sum(c.params for c in costs)
    act = sum(c.act_bytes for c in costs)
    import torch.distributed as dist

    from .. import comm

    held = torch.cuda.memory_allocated() if torch.cuda.is_available() else 0
    # weights + grads, then the saved activations, within 3/4 of what the device has left; the
    # ranks hold different amounts, so they agree on the tightest budget (MIN) before any branch:
    # every rank then takes the same early return or times the chain at the same batch
    budget = _agreed_min(0.75 * hw.hbm_gb * 1e9 - held - nparams * 6)
    if nparams * 6 > 0.25 * hw.hbm_gb * 1e9 or budget <= 0:
        return None
    # halve until it fits: batch / 2^k keeps to the shapes the shipped tuning records hold more
    # often than an arbitrary batch would (every new convolution shape costs an MIOpen search)
    cb = batch
    while cb > 1 and act * cb > budget:
        cb //= 2
    if act * cb > budget:
        return None
    saved = {}
    try:
        t = measure_chain(spine, example_input, costs, batch=cb, dtype=dtype, saved=saved)
    except Exception as e:  # noqa: BLE001 - decided together below
        get_logger().warning("madnn planner: chain timing failed (%s)", e)
        t = None
    if dist.is_initialized() and dist.get_world_size() > 1:
        # all ranks agree before the averaging collective: one failed timing drops it everywhere
        if not comm.all_agree(bool(t), None):
            return None
        v = torch.tensor([t], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(v)   # every GPU timed it: average
        t = float(v) / dist.get_world_size()
    if not t:
        return None
    out = {"batch": batch, "chain_batch": cb, "chain_s": t}
    layers = sum(c.call_s(cb) for c in costs)
    if cb == batch and layers > 0:
        r = t / layers
        for c in costs:
            c.fwd_s *= r
            c.bwd_s *= r
            c.fixed_s *= r
        out.update(ratio=r, layers_s=layers)
    est = act * cb
    if saved.get("bytes", 0) > 0 and est > 0:
        # the meta-device count of bytes written by forward ops includes temporaries that never
        # live until the backward (the fused kernels' internals, views): scale it to the measured
        # saved-activation memory (every rank measured it; ranks agree through the cost broadcast)
        m = min(max(saved["bytes"] / est, 0.05), 2.0)
        for c in costs:
            c.act_bytes *= m
        out["act_ratio"] = m
        out["saved_bytes"] = saved["bytes"]
    return out


def _seg_act(costs, ck, idx) -> float:
    """Saved-activation bytes per sample of the layers ``idx``: a checkpointed layer keeps only
    its boundary tensor, and while one is recomputed its full activations live again (the
    largest checkpointed layer's working set)."""
    kept, work = 0.0, 0.0
    for i in idx:
        if ck[i]:
            kept += costs[i].out_bytes
            work = max(work, costs[i].act_bytes)
        else:
            kept += costs[i].act_bytes
    return kept + work


RECOMPUTE = 1.0 / 3.0   # a checkpointed layer's forward again in the backward: ~1/3 of its fwd + bwd


def _pick_checkpoints(costs, ck, elig, idx, mb, over) -> None:
    """Checkpoint layers of ``idx`` (eligible, not yet chosen) until ``over()`` -- the rank's memory
    above the cap -- is no longer positive, most saved bytes per recompute second first: the
    fewest extra forward seconds for the memory the rank must give up."""
    def gain(i):
        c = costs[i]
        return (c.act_bytes - c.out_bytes) / max(RECOMPUTE * c.call_s(mb), 1e-12)

    for i in sorted((i for i in idx if elig[i] and not ck[i]), key=gain, reverse=True):
        if over() <= 0:
            return
        ck[i] = True


def _candidate(costs, pp, dp, B, cfg, hw: Machine, opt, cap, ckpt, schedule="none", V=1, M=1, elig=None):
    """One placement priced.  ``ckpt``: False (no recompute), True (every eligible layer) or
    "auto" -- per block: on each pipeline rank that would not fit, the fewest eligible layers
    whose recompute makes it fit (``_pick_checkpoints``); None when that equals one of the two
    uniform choices (already priced)."""
    from ..parallel.pp import pipeline_bubble, simulate_schedule, transport_time

    L = len(costs)
    elig = elig if elig is not None else [True] * L
    per_replica = max(B // dp, 1)
    if pp == 1:
        schedule, V, M = "none", 1, 1
    mb = per_replica / M
    ck = [bool(ckpt is True and elig[i]) for i in range(L)]
    nst = pp * V
    pbytes_l = [stage_estimate(costs, i, i + 1, opt, False).param_bytes for i in range(L)]

    def layer_times():
        return [c.call_s(mb) * (1.0 + (RECOMPUTE if ck[i] else 0.0)) for i, c in enumerate(costs)]

    times = layer_times()
    mems = [pbytes_l[i] + _seg_act(costs, ck, [i]) * mb * (pp if pp > 1 else 1) for i in range(L)]
    try:
        bounds, _ = native_runtime.partition(times, nst, mems, cap / V if cap > 0 else 0.0)
    except ValueError:
        bounds, _ = native_runtime.partition(times, nst)
    chunk_est = [stage_estimate(costs, bounds[v], bounds[v + 1], opt, False) for v in range(nst)]
    ranks = _chunk_ranks(pp, V)
    if pp > 1:
        inflight = simulate_schedule(schedule, pp, M, V)["peak_inflight"]
        if schedule == "gpipe":
            inflight = [M * V] * pp
    else:
        inflight = [1]

    def rank_mem(r) -> float:
        vs = ranks[r]
        pbytes = sum(chunk_est[v].param_bytes for v in vs)
        act = sum(_seg_act(costs, ck, range(bounds[v], bounds[v + 1])) for v in vs) / len(vs) * mb
        return pbytes + act * inflight[r]

    if ckpt == "auto":
        for r, vs in enumerate(ranks):
            idx = [i for v in vs for i in range(bounds[v], bounds[v + 1])]
            _pick_checkpoints(costs, ck, elig, idx, mb, lambda r=r: rank_mem(r) - cap)
        k = sum(ck)
        if k == 0 or k == sum(elig):
            return None
        times = layer_times()
    mem_list = [rank_mem(r) / 1e9 for r in range(len(ranks))]
    # per-rank time of ONE microbatch through its chunks: fixed per-call cost + per-sample slope
    rank_t = [sum(times[i] for v in vs for i in range(bounds[v], bounds[v + 1])) for vs in ranks]
    rf = [1.0 + (RECOMPUTE if ck[i] else 0.0) for i in range(L)]
    rb = _reduce_bytes(cfg)
    bucket_bytes = _bucket_bytes(cfg, costs, rb)
    rank_params = [sum(chunk_est[v].params for v in vs) for vs in ranks]
    opt_s = max(optimizer_s(p, opt, hw) for p in rank_params)
    lag = 0.0
    if pp == 1:
        compute = rank_t[0]
        bubble = 0.0
        bwd = [(c.bwd_s * per_replica + c.fixed_s * 2.0 / 3.0) * rf[i] for i, c in enumerate(costs)]
        comm_s = dp_exposed_s(bwd, [c.params * rb for c in costs], dp, hw, bucket_bytes)
        step = compute + comm_s + opt_s
    else:
        compute = M * max(rank_t)
        p2p = max((costs[bounds[v + 1] - 1].out_bytes * mb for v in range(nst - 1)), default=0.0)
        # the engine's transport simulated with this node's (measured) P2P time: bubble AND the
        # transfers the schedule leaves on the critical path
        chunk_s, p2p_s = max(rank_t) / V, hw.p2p_s(p2p)
        pipe = transport_time(schedule, pp, M, V, chunk_s, p2p_s)
        lag = 3.0 * p2p_s / chunk_s if chunk_s > 0 else 0.0   # one transfer in forward-chunk units
        bubble = pipeline_bubble(schedule, pp, M, V)
        comm_s = max(pipe - compute / max(1.0 - bubble, 1e-3), 0.0)   # transfers left on the critical path
        dp_s = 0.0
        if dp > 1:  # stage-local reduction overlaps the last microbatch's backward only
            for vs in ranks:
                idx = [i for v in vs for i in range(bounds[v], bounds[v + 1])]
                bwd = [(costs[i].bwd_s * mb + costs[i].fixed_s * 2.0 / 3.0) * rf[i] for i in idx]
                dp_s = max(dp_s, dp_exposed_s(bwd, [costs[i].params * rb for i in idx], dp, hw, bucket_bytes))
        comm_s += dp_s
        step = pipe + dp_s + opt_s
    fits = max(mem_list) * 1e9 <= cap
    strategy = "dp" if pp == 1 else ("pp" if dp == 1 else "dp_pp")
    return {"strategy": strategy, "dp": dp, "pp": pp, "tp": 1, "M": M, "V": V, "schedule": schedule,
            "ckpt": sum(ck), "ck": ck, "bounds": bounds, "step_s": step, "compute_s": compute, "comm_s": comm_s,
            "bubble": bubble, "mem_gb": max(mem_list), "mem_list": mem_list, "fits": fits, "opt_s": opt_s,
            "lag": lag}


def _tp_linears(layer: nn.Module, tp: int, min_params: int, in_shape, in_dtype):
    """(in, out, tokens per sample) of the Linears ``strategy="tp"`` would shard inside
    ``layer``; tokens come from a META-device forward with hooks on those Linears."""
    mods = [m for m in layer.modules()
            if type(m) is nn.Linear and m.weight.numel() >= min_params and m.in_features % tp == 0]
    if not mods:
        return []
    toks = {}
    hooks = [m.register_forward_hook(lambda mod, inp, out: toks.__setitem__(
        id(mod), int(inp[0].numel() // max(inp[0].shape[-1], 1)))) for m in mods]
    try:
        from torch.func import functional_call

        from .cost import _FlashSDPA, _meta_state

        x = torch.empty((1,) + tuple(in_shape), dtype=in_dtype, device="meta")
        with torch.no_grad(), _FlashSDPA():
            functional_call(layer, _meta_state(layer, None), (x,))
    except Exception:  # noqa: BLE001 - an un-runnable layer: assume one token per sample
        pass
    finally:
        for h in hooks:
            h.remove()
    # a Linear applied functionally (madnn's fused ops.linear) fires no hook: tokens per sample
    # are then the leading dims of the layer input ([S, H] -> S)
    fallback = 1
    for d in tuple(in_shape)[:-1]:
        fallback *= int(d)
    return [(m.in_features, m.out_features, toks.get(id(m), fallback)) for m in mods]


def _tp_candidate(spine: Spine, costs, dp, tp, B, cfg, hw: Machine, opt, cap, example_shape=(), example_dtype=None):
    """dp x tp with row-parallel sharding of the large Linears (``parallel.tp.shard_linears``):
    their GEMM time divides by tp; each adds an output all-reduce (forward) and an input-grad
    all-gather (backward) over the TP group on the critical path."""
    min_params = int(cfg.extra.get("tp_min_params", 1 << 20))
    per_replica = max(B // dp, 1)
    compute = 0.0
    comm = 0.0
    sharded_params = 0
    total_params = sum(c.params for c in costs)
    link_bw = hw.link_gbps * 1e9 * max(min(hw.links, tp - 1), 1) * hw.allreduce_eff
    for i, (layer, c) in enumerate(zip(spine.layers, costs)):
        if i > 0:
            in_shape, in_dtype = costs[i - 1].out_shape, costs[i - 1].out_dtype or torch.float32
        else:
            in_shape, in_dtype = tuple(example_shape), example_dtype
        lin = _tp_linears(layer, tp, min_params, in_shape, in_dtype)
        gflops = sum(2.0 * a * b * t for a, b, t in lin)
        g = min(gflops / c.flops, 1.0) if c.flops > 0 else 0.0
        compute += c.time_s * per_replica * ((1 - g) + g / tp) + c.fixed_s
        for a, b, tokens in lin:
            sharded_params += a * b
            nb_out = tokens * b * 2.0 * per_replica
            nb_in = tokens * a * 2.0 * per_replica
            comm += 2.0 * (tp - 1) / tp * nb_out / link_bw + (tp - 1) / tp * nb_in / link_bw \
                + 2 * hw.collective_latency_us * 1e-6
    if sharded_params == 0:
        return None
    local_params = total_params - sharded_params + sharded_params / tp
    from .cost import param_state_bytes

    act = sum(c.act_bytes for c in costs) * per_replica
    mem = (param_state_bytes(local_params, opt) + act) / 1e9
    grad_dp = 0.0
    if dp > 1:
        bwd = [c.bwd_s * per_replica for c in costs]
        grad_dp = dp_exposed_s(bwd, [c.params * _reduce_bytes(cfg) / tp for c in costs], dp, hw,
                               _bucket_bytes(cfg, costs, _reduce_bytes(cfg)))
    step = compute + comm + grad_dp + optimizer_s(local_params, opt, hw)
    return {"strategy": "tp", "dp": dp, "pp": 1, "tp": tp, "M": 1, "V": 1, "schedule": "none", "ckpt": 0,
            "bounds": [0, len(costs)], "step_s": step, "compute_s": compute, "comm_s": comm + grad_dp,
            "bubble": 0.0, "mem_gb": mem, "mem_list": [mem], "fits": mem * 1e9 <= cap}


__all__ = ["Plan", "plan_model", "trace", "estimate", "infer_example_input", "find_block_list", "dp_exposed_s"]
