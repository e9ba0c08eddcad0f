"""Pipeline-parallel engine (GPipe / 1F1B / interleaved 1F1B) and hybrid DP x PP over RCCL.

Not in the reference ("Pipeline parallel — No"); BASELINE
configs 3 and 4 require it.  Design for one MI355X node:

* one process per GPU; rank -> (dp, pp) coordinates from ``runtime.Mesh``;
  the planner's stage boundaries cut the traced spine into per-rank chunks
  (layers on the META device are materialised only on their own rank, so an
  8B model never exists whole in host memory);
* the per-rank COMPUTE order comes from the C++ scheduler
  (``madnn_pipeline_order``): GPipe, 1F1B, or interleaved 1F1B where every rank
  holds V chunks (virtual stages c*S + rank), shrinking the bubble from
  (S-1)/(M+S-1) toward (S-1)/(V*M+S-1);
* communication is derived from that order (``issue_plan``): every message
  sits in the batch of its producer's finish time on a global schedule clock,
  on both ranks; a batch is at most two ``batch_isend_irecv`` calls (one RCCL
  kernel each): activations on the replica's pipeline communicator, gradients
  on a second one over the same ranks (``P2PTransport``).  Each rank's program
  completes even when every GPU operation of the rank runs one at a time in
  issue order, which is what makes it safe on MI355X, where HIP multiplexes the
  process's streams onto GPU_MAX_HW_QUEUES (4) hardware queues that may
  serialise dispatches of different streams (``simulate_transport`` models the
  queues; ``scripts/hwqueue_probe.py`` measures the sharing).  Two plans --
  boundaries on the compute-only clock and on one with transfer time -- are
  timed in the first steps and the faster is kept.  Reference contrast: the
  reference's collectives are blocking and one at a time
  (datamodule.lua:214-222, nodemodule.lua:52,66,103,117), which cannot deadlock
  but cannot overlap either;
* gradients of each rank are reduced over its DP group by the bucketed
  ``DataParallel`` reducer during each chunk's LAST microbatch backward
  (``no_sync`` before) on links disjoint from the PP hops;
* parameters shared by two ranks (GPT-2's tied ``wte``/``lm_head``) have
  their gradients summed between the owners asynchronously right after the
  last backward; the optimizer updates every other bucket first.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist
from torch import nn
from torch.utils.checkpoint import checkpoint

from .. import comm
from .. import runtime as rt
from ..config import Config
from ..ops import native_runtime, scaled_loss
from ..utils.logging import get_logger
from .dp import DataParallel, _cast_inputs

_DT_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int64: 3}
_CODE_DT = {v: k for k, v in _DT_CODE.items()}


class StageModule(nn.Module):
    """A contiguous run of spine layers, optionally activation-checkpointed per layer."""

    def __init__(self, layers: List[nn.Module], ckpt: Optional[List[bool]] = None):
        super().__init__()
        self.layers = nn.ModuleList(layers)
        self.ckpt = list(ckpt) if ckpt is not None else [False] * len(layers)

    def forward(self, x):
        for layer, c in zip(self.layers, self.ckpt):
            if c and self.training and torch.is_grad_enabled():
                x = checkpoint(layer, x, use_reentrant=False)
            else:
                x = layer(x)
        return x


def materialize_(module: nn.Module, device, init_fn: Optional[Callable] = None, optimizer=None) -> bool:
    """Allocate META parameters/buffers of ``module`` on ``device`` and initialise them.

    ``to_empty`` creates a new Parameter per module slot, which would UNTIE shared weights
    (GPT-2's wte / lm_head); slots that shared one Parameter share the new one again.  An
    ``optimizer`` built over the meta parameters is re-pointed at them (matched by name)."""
    if not any(t.is_meta for t in list(module.parameters()) + list(module.buffers())):
        return False
    old = {id(p): n for n, p in module.named_parameters(remove_duplicate=False)}
    slots: Dict[int, list] = {}
    for m in module.modules():
        for pn, p in m._parameters.items():
            if p is not None:
                slots.setdefault(id(p), []).append((m, pn))
    module.to_empty(device=device)
    for lst in slots.values():
        keep = lst[0][0]._parameters[lst[0][1]]
        for m, pn in lst[1:]:
            m._parameters[pn] = keep
    with torch.no_grad():
        for m in module.modules():
            if init_fn is not None:
                init_fn(m)
            elif hasattr(m, "reset_parameters"):
                m.reset_parameters()
    if optimizer is not None:
        new = dict(module.named_parameters(remove_duplicate=False))
        for g in optimizer.param_groups:
            g["params"] = [new[old[id(p)]] if id(p) in old else p for p in g["params"]]
    return True


def original_names(model: nn.Module, layers: List[nn.Module]):
    """(layer index, local name) -> original-model name for every parameter and buffer of
    ``layers``; computed BEFORE materialisation (which may re-create the tensors)."""
    pid = {}
    for n, p in model.named_parameters(remove_duplicate=False):
        pid.setdefault(id(p), n)
    bid = {}
    for n, b in model.named_buffers(remove_duplicate=False):
        bid.setdefault(id(b), n)
    qual = {id(m): n for n, m in model.named_modules()}
    pmap, bmap = {}, {}
    for i, layer in enumerate(layers):
        q = qual.get(id(layer))
        for n, p in layer.named_parameters(remove_duplicate=False):
            name = pid.get(id(p)) or ((q + "." + n) if q else None)
            if name is not None:
                pmap[(i, n)] = name
        for n, b in layer.named_buffers(remove_duplicate=False):
            name = bid.get(id(b)) or ((q + "." + n) if q else None)
            if name is not None:
                bmap[(i, n)] = name
    return pmap, bmap


def stage_names(layers: List[nn.Module], pmap, bmap):
    """Resolve the (layer, local name) maps against the (possibly re-created) stage tensors."""
    pnames: Dict[int, str] = {}
    bufs = []
    for i, layer in enumerate(layers):
        for n, p in layer.named_parameters(remove_duplicate=False):
            if (i, n) in pmap:
                pnames.setdefault(id(p), pmap[(i, n)])
        seen = set()
        for n, _ in layer.named_buffers(remove_duplicate=False):
            if (i, n) in bmap and bmap[(i, n)] not in seen:
                seen.add(bmap[(i, n)])
                bufs.append((bmap[(i, n)], layer, n))
    return pnames, bufs


def restrict_optimizer(opt, params: List[nn.Parameter]):
    """A new optimizer of the same type/hyper-parameters over ``params`` only."""
    keep = {id(p) for p in params}
    groups = []
    for g in opt.param_groups:
        ps = [p for p in g["params"] if id(p) in keep]
        if ps:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = ps
            groups.append(d)
    if not groups:
        groups = [{"params": params}]
    # the constructor's own keyword arguments only: a torch optimizer's defaults can carry derived
    # entries it does not accept back (AdamW: decoupled_weight_decay); the groups keep every value
    import inspect

    sig = inspect.signature(type(opt).__init__).parameters
    kw = {k: v for k, v in opt.defaults.items() if k in sig}
    return type(opt)(groups, **kw)


# ----------------------------------------------------------------------------
# schedule analysis (pure Python; also used by the planner to price the bubble)
# ----------------------------------------------------------------------------
def virtual_stage(chunk: int, stage: int, nstages: int) -> int:
    """Chunk ``chunk`` of pipeline rank ``stage`` is virtual stage chunk*S + stage."""
    return chunk * nstages + stage


def simulate_schedule(kind: str, nstages: int, nmicro: int, nchunks: int = 1, t_fwd: float = 1.0,
                      t_bwd: float = 2.0, t_p2p: float = 0.0) -> dict:
    """Execute every rank's compute order (``native_runtime.pipeline_order``) against
    one-directional FIFO channels with non-blocking sends, as the engine does.

    Raises RuntimeError if the schedule deadlocks or a channel's receive order differs from
    its send order (the property that lets the engine post receives ahead of time).  Returns
    ``{"makespan", "bubble", "peak_inflight"}`` for per-chunk forward/backward costs
    ``t_fwd``/``t_bwd`` and a per-message latency ``t_p2p``; ``bubble`` is the idle fraction
    of the busiest rank (the analytic (S-1)/(M+S-1) for 1F1B, less when interleaved)."""
    S, M, V = nstages, nmicro, nchunks
    SV = S * V
    orders = [native_runtime.pipeline_order(kind, s, S, M, V) for s in range(S)]
    done: Dict[tuple, float] = {}          # (op, vs, m) -> finish time
    began: Dict[tuple, float] = {}         # (op, vs, m) -> start time
    sent: Dict[tuple, list] = {}           # channel -> list of messages in send order
    recv_seq: Dict[tuple, list] = {}       # channel -> list of messages in consume order
    pos = [0] * S
    free = [0.0] * S
    busy = [0.0] * S
    live = [0] * S
    peak = [0] * S

    def chan(kind_, src_vs, dst_vs):
        return (kind_, src_vs % S, dst_vs % S)

    total = sum(len(o) for o in orders)
    finished = 0
    while finished < total:
        progressed = False
        for s in range(S):
            while pos[s] < len(orders[s]):
                op, c, m = orders[s][pos[s]]
                vs = c * S + s
                if op == "F":
                    dep = ("F", vs - 1, m) if vs > 0 else None
                else:
                    dep = ("B", vs + 1, m) if vs < SV - 1 else ("F", vs, m)
                if dep is not None and dep not in done:
                    break
                ready = done[dep] + (t_p2p if dep[1] != vs else 0.0) if dep is not None else 0.0
                start = max(free[s], ready)
                dur = t_fwd if op == "F" else t_bwd
                free[s] = start + dur
                busy[s] += dur
                done[(op, vs, m)] = free[s]
                began[(op, vs, m)] = start
                if op == "F":
                    live[s] += 1
                    peak[s] = max(peak[s], live[s])
                    if vs > 0:
                        recv_seq.setdefault(chan("act", vs - 1, vs), []).append((vs, m))
                    if vs < SV - 1:
                        sent.setdefault(chan("act", vs, vs + 1), []).append((vs + 1, m))
                else:
                    live[s] -= 1
                    if vs < SV - 1:
                        recv_seq.setdefault(chan("grad", vs + 1, vs), []).append((vs, m))
                    if vs > 0:
                        sent.setdefault(chan("grad", vs, vs - 1), []).append((vs - 1, m))
                pos[s] += 1
                finished += 1
                progressed = True
        if not progressed:
            stuck = {s: orders[s][pos[s]] for s in range(S) if pos[s] < len(orders[s])}
            raise RuntimeError(f"pipeline schedule {kind} S={S} M={M} V={V} deadlocks at {stuck}")
    for ch, msgs in sent.items():
        if recv_seq.get(ch, []) != msgs:
            raise RuntimeError(f"channel {ch}: receive order differs from send order")
    makespan = max(free)
    return {"makespan": makespan, "bubble": 1.0 - max(busy) / makespan, "peak_inflight": peak,
            "times": {k: (began[k], done[k]) for k in done}}


# ----------------------------------------------------------------------------
# issue plan: the per-rank program of compute and batched P2P exchanges
# ----------------------------------------------------------------------------
_TIMELINE_CACHE: Dict[tuple, dict] = {}


def _timeline(kind: str, nstages: int, nmicro: int, nchunks: int, lag: float = 0.0) -> dict:
    key = (kind, nstages, nmicro, nchunks, lag)
    if key not in _TIMELINE_CACHE:
        _TIMELINE_CACHE[key] = simulate_schedule(kind, nstages, nmicro, nchunks, t_p2p=lag)["times"]
    return _TIMELINE_CACHE[key]


# transfer time in forward-chunk units the engine's second issue plan assumes when the plan
# carries none (a hand-written placement): GPT-2 medium's 8-GPU plan prices 0.27-0.8
_DEFAULT_LAG = 0.3


def _planned_lag(plan) -> float:
    """The issue-plan lag the planner priced; the default only when the plan carries none (a
    planned 0.0 -- transfers priced as negligible -- stays 0: no second plan to time)."""
    lag = getattr(plan, "p2p_lag", None)
    return _DEFAULT_LAG if lag is None else float(lag)


def plan_lag(lag: float) -> float:
    """A transfer time in forward-chunk units, rounded to 2 significant digits (the issue plans
    and their caches are keyed on it)."""
    return float(f"{lag:.2g}") if lag > 0 else 0.0


def issue_plan(kind: str, stage: int, nstages: int, nmicro: int, nchunks: int = 1,
               lag: float = 0.0) -> List[tuple]:
    """The program one pipeline rank issues per step: ``("C", op, c, m)`` compute items and
    ``("X", ops)`` point-to-point batches, ``ops`` = ``(("send"|"recv", "act"|"grad", c, m, peer
    stage), ...)``.  The engine issues each batch as ONE ``batch_isend_irecv`` on the replica's
    pipeline communicator (one ncclGroup: one kernel per batch) and orders the compute that
    consumes a received tensor after it.

    Construction (any compute order: GPipe, 1F1B, interleaved): a schedule of the computes
    (:func:`simulate_schedule`, forward 1 / backward 2, each transfer ``lag`` forward-units long)
    gives every compute a start and a finish time on one global clock.  Each message is assigned to the BOUNDARY at its producer's
    finish time T, on both ranks: the sender issues it right after the producer, the receiver
    in a batch placed before its first compute that starts at or after T (a compute that
    started earlier goes first).  Messages of one rank with the same boundary share a batch; in
    balanced 1F1B that is exactly Megatron-LM's ``send_forward_recv_backward`` /
    ``send_backward_recv_forward`` pairing.  A batch that only receives is issued from an idle
    side stream, so its transfer does not wait for the compute issued before it (RCCL orders a
    kernel after all work of the stream current at issue time).

    Why: every rank's program then completes even when ALL of its GPU work -- computes, these
    batch kernels, the DP all-reduce, the tied-gradient sum -- runs one operation at a time in
    issue order, and a send completes only together with its receive (rendezvous).  By
    induction over the boundaries in time order, every rank reaches its batch of boundary T
    (everything before it needs only messages of earlier boundaries), and the batches of one
    boundary name exactly each other's messages.  HIP multiplexes a process's streams onto
    GPU_MAX_HW_QUEUES (4) hardware queues, whose dispatches can serialise across streams
    (``scripts/hwqueue_probe.py``); such sharing only ADDS ordering to a program that already
    completes fully serialised, and an operation that could run stays runnable until it does,
    so no stream-to-queue mapping can deadlock it (:func:`simulate_transport` checks
    ``queues="serial"``, round-robin queue pools and independent queues).  The round-3 engine
    pre-posted every receive of the step, which deadlocks as soon as one of those spinning
    receive kernels shares a queue with the compute stream (``design="prepost"``).

    ``lag``: the argument holds for ANY consistent clock, so the transfer time can be part of
    it.  With ``lag`` > 0 a receiver's batch lands before its first compute that starts after
    the producer finished -- earlier relative to the consumer than with ``lag`` = 0, which lets
    an interleaved schedule's slack hide the transfer (``simulate_transport`` with independent
    queues: S = 4, M = 16, V = 2 at transfers of 0.27 forward: 108.9 vs 118.5, the round-3
    pre-posting's 108.8) -- but a receive posted earlier also holds its hardware queue longer, so
    when the gradient communicator shares the compute stream's queue ``lag`` = 0 is better
    (123.4 vs 168.1).  The engine measures both on the job and keeps the faster."""
    S, V = nstages, nchunks
    SV = S * V
    order = native_runtime.pipeline_order(kind, stage, S, nmicro, V)
    times = _timeline(kind, S, nmicro, V, plan_lag(lag))
    items: List[tuple] = []
    batches: Dict[float, list] = {}
    for op, c, m in order:
        vs = c * S + stage
        start, finish = times[(op, vs, m)]
        items.append(((start, 1), ("C", op, c, m)))
        if op == "F":
            if vs > 0:
                batches.setdefault(times[("F", vs - 1, m)][1], []).append(("recv", "act", c, m, (stage - 1) % S))
            if vs < SV - 1:
                batches.setdefault(finish, []).append(("send", "act", c, m, (stage + 1) % S))
        else:
            if vs < SV - 1:
                batches.setdefault(times[("B", vs + 1, m)][1], []).append(("recv", "grad", c, m, (stage + 1) % S))
            if vs > 0:
                batches.setdefault(finish, []).append(("send", "grad", c, m, (stage - 1) % S))
    for t, ops in batches.items():
        items.append(((t, 0), ("X", tuple(sorted(ops, key=lambda o: (o[0] != "send", o[4], o[1]))))))
    items.sort(key=lambda kv: kv[0])
    return [it for _, it in items]


def _message(d: str, kind: str, c: int, m: int, stage: int, nstages: int) -> tuple:
    """Global identity of a P2P message: (kind, receiving virtual stage, microbatch)."""
    vs = c * nstages + stage
    if d == "recv":
        return (kind, vs, m)
    return (kind, vs + 1 if kind == "act" else vs - 1, m)


def check_plan_fifo(kind: str, nstages: int, nmicro: int, nchunks: int = 1, lag: float = 0.0) -> int:
    """Every ordered rank pair's messages are received in the order they are sent (the
    communicator matches P2P operations of one pair FIFO).  Returns the message count; raises
    RuntimeError on a mismatch (which would deliver one microbatch's data to another)."""
    S = nstages
    sent: Dict[tuple, list] = {}
    recvd: Dict[tuple, list] = {}
    for s in range(S):
        for item in issue_plan(kind, s, S, nmicro, nchunks, lag):
            if item[0] != "X":
                continue
            for d, k, c, m, peer in item[1]:
                msg = _message(d, k, c, m, s, S)
                if d == "send":
                    sent.setdefault((s, peer), []).append(msg)
                else:
                    recvd.setdefault((peer, s), []).append(msg)
    for pair in set(sent) | set(recvd):
        if sent.get(pair, []) != recvd.get(pair, []):
            raise RuntimeError(f"pipeline plan {kind} S={S} M={nmicro} V={nchunks}: pair {pair} receives "
                               f"{recvd.get(pair)} but is sent {sent.get(pair)}")
    return sum(len(v) for v in sent.values())


def recv_plan(order, vstages: List[int], nvirtual: int) -> List[tuple]:
    """Every receive of one pipeline rank's step in issue order (``("act", c, m)`` before the
    forward of a non-first virtual stage, ``("grad", c, m)`` before the backward of a non-last
    one): what the round-3 engine pre-posted at step start.  Kept for the transport model."""
    out = []
    for op, c, m in order:
        vs = vstages[c]
        if op == "F" and vs > 0:
            out.append(("act", c, m))
        elif op == "B" and vs < nvirtual - 1:
            out.append(("grad", c, m))
    return out


def rank_streams(design: str, stage: int, nstages: int, dp: int = 1, tied: bool = False,
                 nchunks: int = 1) -> List[str]:
    """The HIP streams one pipeline rank drives, in creation order (the order in which HIP hands
    out hardware queues): the compute (default) stream, one RCCL stream per communicator the
    rank uses -- WORLD from ``init_process_group``, the mesh axis groups in ``AXES`` order with
    singleton axes skipped (the pipeline group carries the activations; with dp == 1 it is
    WORLD), the replica's gradient group (``split``), the tied-parameter group, the round-3
    per-channel groups (``prepost``) -- and madnn's DP comm stream."""
    S = nstages
    out = ["compute", "world"]
    if dp > 1:
        out.append("dp")
    if dp > 1:          # with dp == 1 the pipeline group IS the world group
        out.append("pp")
    if design == "split":
        out.append("p2p_grad")
    if tied and S > 1 and stage in (0, S - 1):
        out.append("tied")
    if design == "prepost":
        edges = [(e, e + 1) for e in range(S - 1)] + [(e + 1, e) for e in range(S - 1)]
        if nchunks > 1:
            edges += [(S - 1, 0), (0, S - 1)]
        out += [f"chan{a}-{b}" for a, b in edges if stage in (a, b)]
    out.append("dpcomm")
    return out


def simulate_transport(kind: str, nstages: int, nmicro: int, nchunks: int = 1, design: str = "split",
                       queues=None, dp: int = 1, tied: bool = False, first_step: bool = False,
                       queue_offset: int = 0, t_fwd: float = 1.0, t_bwd: float = 2.0, t_p2p: float = 0.0,
                       t_coll: float = 0.0, lag: float = 0.0) -> dict:
    """Replay one training step of every rank of a ``dp x nstages`` pipeline mesh against a model
    of the GPU's execution: every HIP stream of a rank feeds a hardware queue, and a queue runs
    its operations ONE AT A TIME in submission order (a compute kernel for ``t_fwd``/``t_bwd``, an
    event wait blocks the queue until its event, a communication kernel occupies the queue until
    it completes).

    ``queues``: ``None`` -- every stream its own queue; ``"serial"`` -- one queue per rank (every
    operation of the rank serialised: the strongest constraint); an int Q -- stream i of
    :func:`rank_streams` (creation order) on queue ``(i + queue_offset) % Q``, the round-robin
    assignment HIP uses for a pool of Q hardware queues.

    Communication follows RCCL: a batch kernel moves each of its messages once the matching
    kernel on the peer is running too (rendezvous; the batch completes with its last message);
    a collective completes once every member runs it; a kernel issued while a stream with
    pending work is current waits for that work (ProcessGroupNCCL's stream sync).
    ``design``: ``"split"`` is the engine (:func:`issue_plan`; each batch's activation part on
    the replica's pipeline communicator and its gradient part on a second one; a part that only
    receives is issued from an idle side stream, one that sends after the producing compute;
    the consumer waits for its part; the DP all-reduce of each chunk's buckets on the dp
    communicator during its last microbatch backward; the tied-gradient sum between the first
    and last stage after the step); ``"batched"`` is the same plan on ONE communicator;
    ``"prepost"`` is the round-3 engine (one 2-rank communicator per channel, every receive of
    the step posted up front).  ``first_step`` adds the shape headers a new input signature
    exchanges (host-blocking).  ``lag``: the issue plan's transfer time (:func:`issue_plan`).

    Raises RuntimeError on a deadlock (naming every stuck queue head) or a FIFO mismatch;
    returns ``{"makespan", "bubble", "ops", "queues"}``."""
    S, M, V = nstages, nmicro, nchunks
    SV = S * V
    if design not in ("batched", "split", "prepost"):
        raise ValueError(f"unknown transport design {design!r}")
    ranks = [(d, s) for d in range(dp) for s in range(S)]
    rid = {r: i for i, r in enumerate(ranks)}
    ops: List[dict] = []
    programs: List[list] = []
    streams = [rank_streams(design, s, S, dp, tied, V) for (_d, s) in ranks]
    pstream = "pp" if dp > 1 else "world"   # with dp == 1 the pipeline group is the world group

    def new(kind_, r, stream, deps=(), **kw):
        ops.append(dict(kind=kind_, rank=r, stream=stream, deps=[x for x in deps if x is not None], start=None,
                        done=None, **kw))
        return len(ops) - 1

    sends: Dict[tuple, list] = {}   # (src, dst) -> [(op id, message)] in issue order
    recvs: Dict[tuple, list] = {}

    def xfer(oid, d, k, c, m, s, peer_stage, r, drep):
        msg = _message(d, k, c, m, s, S) if k in ("act", "grad") else (k, c, m)
        peer = rid[(drep, peer_stage)]
        if d == "send":
            sends.setdefault((r, peer), []).append((oid, msg))
        else:
            recvs.setdefault((peer, r), []).append((oid, msg))

    for (d, s) in ranks:
        r = rid[(d, s)]
        prog = []
        if design in ("batched", "split"):
            last_c = None
            need = None
            met_in, met_out = set(), set()
            for item in issue_plan(kind, s, S, M, V, lag):
                if item[0] == "X":
                    batch = item[1]
                    if first_step:
                        hdr = [(dd, k, c, m, p) for dd, k, c, m, p in batch if k == "act" and
                               ((dd == "recv" and c not in met_in) or (dd == "send" and c not in met_out))]
                        if hdr:
                            h = new("X", r, pstream, [last_c])
                            for dd, k, c, m, p in hdr:
                                (met_in if dd == "recv" else met_out).add(c)
                                xfer(h, dd, "hdr", _message(dd, k, c, m, s, S)[1], m, s, p, r, d)
                            prog += [("issue", h), ("hostwait", h)]
                    if design == "batched":
                        parts = [(pstream, batch)]
                    else:                  # the engine: activations and gradients on two communicators
                        parts = [(pstream if k == "act" else "p2p_grad", tuple(o for o in batch if o[1] == k))
                                 for k in ("act", "grad")]
                    for stream_name, part in parts:
                        if not part:
                            continue
                        has_send = any(o[0] == "send" for o in part)
                        x = new("X", r, stream_name, [last_c] if has_send else [], desc=part)
                        for dd, k, c, m, p in part:
                            xfer(x, dd, k, c, m, s, p, r, d)
                        prog.append(("issue", x))
                        if any(dd == "recv" for dd, *_ in part):
                            need = x
                else:
                    _, op, c, m = item
                    vs = c * S + s
                    takes = (op == "F" and vs > 0) or (op == "B" and vs < SV - 1)
                    last_c = new("C", r, "compute", [need] if takes else [], dur=t_fwd if op == "F" else t_bwd,
                                 desc=(op, c, m))
                    prog.append(("issue", last_c))
                    if takes:
                        need = None
                    if op == "B" and m == M - 1 and dp > 1:
                        a = new("A", r, "dp", [last_c], key=("dp", s, c), members=[rid[(e, s)] for e in range(dp)])
                        prog.append(("issue", a))
            if tied and S > 1 and s in (0, S - 1):
                a = new("A", r, "tied", [last_c], key=("tied", d), members=[rid[(d, 0)], rid[(d, S - 1)]])
                prog.append(("issue", a))
        else:  # prepost: the round-3 engine
            order = native_runtime.pipeline_order(kind, s, S, M, V)
            vst = [virtual_stage(c, s, S) for c in range(V)]
            rec = {}
            for k, c, m in recv_plan(order, vst, SV):
                peer = (s - 1) % S if k == "act" else (s + 1) % S
                oid = new("X", r, f"chan{peer}-{s}")
                xfer(oid, "recv", k, c, m, s, peer, r, d)
                rec[(k, c, m)] = oid
                prog.append(("issue", oid))
            last_c = None
            for op, c, m in order:
                vs = vst[c]
                key = ("act", c, m) if op == "F" and vs > 0 else (("grad", c, m) if op == "B" and vs < SV - 1 else None)
                last_c = new("C", r, "compute", [rec[key]] if key else [], dur=t_fwd if op == "F" else t_bwd)
                prog.append(("issue", last_c))
                if op == "F" and vs < SV - 1:
                    peer = (s + 1) % S
                    oid = new("X", r, f"chan{s}-{peer}", [last_c])
                    xfer(oid, "send", "act", c, m, s, peer, r, d)
                    prog.append(("issue", oid))
                elif op == "B" and vs > 0:
                    peer = (s - 1) % S
                    oid = new("X", r, f"chan{s}-{peer}", [last_c])
                    xfer(oid, "send", "grad", c, m, s, peer, r, d)
                    prog.append(("issue", oid))
                if op == "B" and m == M - 1 and dp > 1:
                    prog.append(("issue", new("A", r, "dp", [last_c], key=("dp", s, c),
                                              members=[rid[(e, s)] for e in range(dp)])))
            if tied and S > 1 and s in (0, S - 1):
                prog.append(("issue", new("A", r, "tied", [last_c], key=("tied", d),
                                          members=[rid[(d, 0)], rid[(d, S - 1)]])))
        programs.append(prog)

    # pair the k-th send of every ordered rank pair with the k-th receive (communicator FIFO)
    xfers: List[list] = []          # transfer id -> [sender op, receiver op]
    for pair in set(sends) | set(recvs):
        a, b = sends.get(pair, []), recvs.get(pair, [])
        if [msg for _, msg in a] != [msg for _, msg in b]:
            raise RuntimeError(f"transport {design} {kind} S={S} M={M} V={V}: pair {pair} sends "
                               f"{[msg for _, msg in a]} but receives {[msg for _, msg in b]}")
        for (so, _), (ro, _) in zip(a, b):
            tid = len(xfers)
            xfers.append([so, ro])
            ops[so].setdefault("xfers", []).append(tid)
            ops[ro].setdefault("xfers", []).append(tid)
    xdone: Dict[int, float] = {}
    coll: Dict[tuple, list] = {}
    for i, o in enumerate(ops):
        if o["kind"] == "A":
            coll.setdefault(o["key"], []).append(i)

    def qid(r, stream):
        if queues is None:
            return stream
        if queues == "serial":
            return 0
        return (streams[r].index(stream) + queue_offset) % int(queues)

    pc = [0] * len(ranks)
    fifo: Dict[tuple, list] = {}
    qfree: Dict[tuple, float] = {}
    busy = [0.0] * len(ranks)
    remaining = len(ops)
    while remaining:
        progressed = False
        for r, prog in enumerate(programs):        # the host issues until an unfinished host wait
            while pc[r] < len(prog):
                what, oid = prog[pc[r]]
                if what == "hostwait":
                    if ops[oid]["done"] is None:
                        break
                else:
                    fifo.setdefault((r, qid(r, ops[oid]["stream"])), []).append(oid)
                pc[r] += 1
                progressed = True
        for q, lst in fifo.items():
            while lst:
                o = ops[lst[0]]
                if o["done"] is None:
                    if o["start"] is None:
                        if any(ops[x]["done"] is None for x in o["deps"]):
                            break
                        o["start"] = max([qfree.get(q, 0.0)] + [ops[x]["done"] for x in o["deps"]])
                        progressed = True
                    if o["kind"] == "C":
                        o["done"] = o["start"] + o["dur"]
                        busy[o["rank"]] += o["dur"]
                    elif o["kind"] == "X":
                        for tid in o.get("xfers", []):
                            if tid in xdone:
                                continue
                            other = ops[xfers[tid][0] if xfers[tid][1] == lst[0] else xfers[tid][1]]
                            if other["start"] is not None:
                                xdone[tid] = max(o["start"], other["start"]) + t_p2p
                        if any(tid not in xdone for tid in o.get("xfers", [])):
                            break
                        o["done"] = max([o["start"]] + [xdone[t] for t in o.get("xfers", [])])
                    else:
                        members = [ops[x] for x in coll[o["key"]]]
                        if any(mo["start"] is None for mo in members):
                            break
                        end = max(mo["start"] for mo in members) + t_coll
                        for mo in members:
                            mo["done"] = end
                qfree[q] = o["done"]
                lst.pop(0)
                remaining -= 1
                progressed = True
        if not progressed:
            heads = {}
            for (r, q), lst in fifo.items():
                if lst:
                    o = ops[lst[0]]
                    heads.setdefault(ranks[r], []).append((q, o["stream"], o["kind"], o.get("key") or o.get("desc")))
            raise RuntimeError(f"pipeline transport {design} {kind} S={S} M={M} V={V} dp={dp} queues={queues} "
                               f"deadlocks; queue heads: {heads}")
    makespan = max(o["done"] for o in ops)
    return {"makespan": makespan, "bubble": 1.0 - max(busy) / makespan if makespan else 0.0, "ops": len(ops),
            "queues": queues}


# ----------------------------------------------------------------------------
# transport
# ----------------------------------------------------------------------------
def _emulated_p2p_timeout() -> Optional[float]:
    import os

    v = os.environ.get("MADNN_EMULATE_RCCL_P2P", "")
    if v in ("", "0"):
        return None
    return float(os.environ.get("MADNN_EMULATE_RCCL_P2P_TIMEOUT", "60"))


class P2PTransport:
    """The point-to-point exchanges of one pipeline replica on TWO communicators: activations on
    the replica's pipeline group (WORLD when dp == 1), gradients on a second group over the same
    ranks -- so in 1F1B's steady state the gradient a rank waits for never queues behind the
    activation it just sent (``simulate_transport``: ``split`` vs ``batched``).

    :meth:`exchange` issues one :func:`issue_plan` batch: per kind one ``batch_isend_irecv``
    (on RCCL one ncclGroup: one kernel moving every message of that part, whichever peer it
    goes to).  A part that sends is issued on the current (compute) stream, after the producer;
    a part that only receives is issued from an idle side stream, so its kernel does not wait
    for the compute issued before it and the transfer overlaps that compute.  The current
    stream is then ordered after every part that received (a stream wait, no host block);
    send-only parts are waited for at the end of the step (:meth:`drain`).

    On a gloo group HIP tensors are staged through host memory (several ranks on one GPU in
    tests; RCCL refuses that).  ``MADNN_EMULATE_RCCL_P2P=1`` makes the CPU tests execute every
    part the way the strongest hardware-queue model does (``simulate_transport`` with
    ``queues="serial"``): the part first rendezvouses with every peer it names (a token
    exchange), then moves its data, and the host waits for it -- one operation at a time per
    rank; a wait that outlasts ``MADNN_EMULATE_RCCL_P2P_TIMEOUT`` is reported as a transport
    deadlock."""

    def __init__(self, act_group, grad_group, stage_ranks: List[int], device):
        self.groups = {"act": act_group, "grad": grad_group}
        self.stage_ranks = list(stage_ranks)
        self.device = torch.device(device)
        backend = dist.get_backend(act_group) if dist.is_initialized() else "gloo"
        self.staged = backend == "gloo" and self.device.type == "cuda"
        self.buf_device = torch.device("cpu") if self.staged else self.device
        self.emulate = _emulated_p2p_timeout() if backend == "gloo" else None
        self.side = torch.cuda.Stream(self.device) if backend == "nccl" and self.device.type == "cuda" else None
        self._inflight = []        # (works, tensors kept alive) of send-only parts not waited for yet
        self._keep = []            # sent tensors of parts already waited for (alive until drain)
        self._seq: Dict[tuple, int] = {}   # emulation: per (kind, direction, peer) message count
        self.bytes = 0
        self.messages = 0
        self.batches = 0

    def _wait(self, works):
        if self.emulate is None:
            for w in works:
                w.wait()
            return
        import datetime

        for w in works:
            try:
                ok = w.wait(timeout=datetime.timedelta(seconds=self.emulate))
            except RuntimeError as e:
                raise RuntimeError(f"emulated RCCL P2P: batch not complete after {self.emulate:.0f} s "
                                   f"(transport deadlock): {e}") from e
            if ok is False:
                raise RuntimeError(f"emulated RCCL P2P: batch not complete after {self.emulate:.0f} s "
                                   "(transport deadlock)")

    def exchange(self, sends, recvs, kind: str = "act") -> List[torch.Tensor]:
        """One part on the ``kind`` communicator: ``sends`` = [(tensor, peer stage)], ``recvs`` =
        [(shape, dtype, peer stage)].  Returns the received tensors on the compute device,
        ordered after the part."""
        group = self.groups[kind]
        ops, keep, bufs = [], [], []
        for t, peer in sends:
            t = t.detach().contiguous()
            if self.staged:
                t = t.cpu()
            keep.append(t)
            comm._record("send", group, t)
            ops.append(dist.P2POp(dist.isend, t, self.stage_ranks[peer], group))
            self.bytes += t.numel() * t.element_size()
            self.messages += 1
        side = self.side is not None and not sends and self.emulate is None
        for shape, dtype, peer in recvs:
            if side:
                # a receive-only part runs unordered with the compute stream, so its buffer must
                # not come from blocks the compute stream freed but may still be reading: allocate
                # it on the side stream (record_stream below hands it to the compute stream)
                with torch.cuda.stream(self.side):
                    b = torch.empty(shape, dtype=dtype, device=self.buf_device)
            else:
                b = torch.empty(shape, dtype=dtype, device=self.buf_device)   # ordered after the producer
            comm._record("recv", group, b)
            bufs.append(b)
            ops.append(dist.P2POp(dist.irecv, b, self.stage_ranks[peer], group))
        if not ops:
            return []
        self.batches += 1
        if self.emulate is not None:
            self._rendezvous(kind, group, [p for _, p in sends], [p for *_, p in recvs])
            self._wait(dist.batch_isend_irecv(ops))
        else:
            if side:
                # receive only: issue from the idle side stream (no wait on the compute queued so far)
                with torch.cuda.stream(self.side):
                    works = dist.batch_isend_irecv(ops)
            else:
                works = dist.batch_isend_irecv(ops)
            if bufs:
                self._wait(works)      # RCCL: the current stream waits for the part's kernel
                if side:
                    cur = torch.cuda.current_stream(self.device)
                    for b in bufs:
                        b.record_stream(cur)
                if keep:
                    self._keep.append(keep)
            else:
                # never wait twice: a second wait on a finished gloo receive blocks for a new one
                self._inflight.append((works, keep))
        return [b.to(self.device, non_blocking=False) if self.staged else b for b in bufs]

    def exchange_batch(self, sends, recvs) -> List[torch.Tensor]:
        """A whole :func:`issue_plan` batch: ``sends`` = [(kind, tensor, peer)], ``recvs`` =
        [(kind, shape, dtype, peer)]; the activation part first, then the gradient part (the
        order :func:`simulate_transport` verifies).  Returns the received tensors in ``recvs``
        order."""
        out = {}
        for kind in ("act", "grad"):
            idx = [i for i, r in enumerate(recvs) if r[0] == kind]
            got = self.exchange([(t, p) for k, t, p in sends if k == kind],
                                [recvs[i][1:] for i in idx], kind)
            out.update(zip(idx, got))
        return [out[i] for i in range(len(recvs))]

    def _rendezvous(self, kind, group, send_peers, recv_peers):
        """Emulation only: meet every peer of this part and check that the peer's current part
        carries exactly the complementary messages (by per-pair FIFO sequence number) -- the
        condition for an RCCL batch kernel to finish while both ranks run one operation at a
        time.  A mismatch is the deadlock the real transport would hang in; it raises here."""
        me = self.stage_ranks.index(dist.get_rank()) if dist.get_rank() in self.stage_ranks else -1
        mine: Dict[int, list] = {}
        for p in send_peers:
            k = self._seq.get((kind, "s", p), 0)
            self._seq[(kind, "s", p)] = k + 1
            mine.setdefault(p, []).append((me, p, k))
        for p in recv_peers:
            k = self._seq.get((kind, "r", p), 0)
            self._seq[(kind, "r", p)] = k + 1
            mine.setdefault(p, []).append((p, me, k))
        peers = sorted(mine)
        tok = [torch.tensor([hash(tuple(sorted(mine[p]))) & 0x7FFFFFFFFFFF], dtype=torch.int64) for p in peers]
        got = [torch.zeros(1, dtype=torch.int64) for _ in peers]
        ops = []
        for p, t, g in zip(peers, tok, got):
            ops.append(dist.P2POp(dist.isend, t, self.stage_ranks[p], group))
            ops.append(dist.P2POp(dist.irecv, g, self.stage_ranks[p], group))
        self._wait(dist.batch_isend_irecv(ops))
        for p, t, g in zip(peers, tok, got):
            if int(t) != int(g):
                raise RuntimeError(f"emulated RCCL P2P: transport deadlock: stage {me} and stage {p} are in "
                                   f"different {kind} batches (this side moves {sorted(mine[p])})")

    def exchange_meta(self, sends, recv_peers) -> List[tuple]:
        """Activation shape headers for the first step of an input signature: ``sends`` =
        [(tensor, peer stage)] announce their shape/dtype; returns ``(shape, dtype)`` per entry of
        ``recv_peers``.  Host-blocking (the receiver must size its buffer)."""
        hdrs = []
        for t, peer in sends:
            h = torch.zeros(10, dtype=torch.int64)
            h[0] = t.dim()
            h[1] = _DT_CODE[t.dtype]
            h[2:2 + t.dim()] = torch.tensor(t.shape, dtype=torch.int64)
            hdrs.append((h.to(self.buf_device), peer))
        got = self.exchange(hdrs, [((10,), torch.int64, p) for p in recv_peers], "act")
        out = []
        for g in got:
            v = g.tolist()
            out.append((tuple(int(x) for x in v[2:2 + v[0]]), _CODE_DT[v[1]]))
        return out

    def drain(self) -> None:
        """Order the current stream after every part of this step (RCCL) / wait for them (gloo)."""
        for works, _keep in self._inflight:
            self._wait(works)
        self._inflight.clear()
        self._keep.clear()


# ----------------------------------------------------------------------------
# engine
# ----------------------------------------------------------------------------
class PipelineStage(nn.Module):
    """The model chunks one pipeline rank holds (one per virtual stage)."""

    def __init__(self, chunks: List[StageModule]):
        super().__init__()
        self.chunks = nn.ModuleList(chunks)

    def forward(self, x, chunk: int = 0):
        return self.chunks[chunk](x)


class PipelineEngine:
    """Runs one pipeline rank of a (dp x pp) mesh; ``train_step`` = fwd + bwd of all microbatches.

    The compute order comes from the C++ scheduler (GPipe, 1F1B or interleaved 1F1B with V
    chunks per rank) and the rank executes :func:`issue_plan` of it: between two computes, one
    batched exchange with the neighbours (the activation of the previous forward out, the input
    of the next compute in), on the replica's pipeline communicator (the ring edge S-1 -> 0
    carries activations between chunks when V > 1).  Every program is deadlock-free even fully
    serialised, so no sharing of the GPU's hardware queues between its streams can stall it
    (:func:`simulate_transport`).  The first step of an input signature exchanges shape headers
    just before the data batches that need them."""

    def __init__(self, stage_module: PipelineStage, *, stage: int, nstages: int, groups: rt.ProcessGroups,
                 microbatches: int, schedule: str, loss_fn: Callable, dp_engine: DataParallel,
                 cast_dtype, tied: List[tuple], param_names: Dict[int, str], buffer_refs=(),
                 transport: Optional[P2PTransport] = None, lag: float = 0.0, sig_group=None):
        self.module = stage_module
        self.chunks = list(stage_module.chunks)
        self.V = len(self.chunks)
        self.stage, self.nstages = stage, nstages
        self.groups = groups
        self.M = microbatches
        self.schedule = schedule
        self.loss_fn = loss_fn
        self.dp = dp_engine
        self.dp.defer_flush = True          # the engine launches the leftover buckets after the LAST backward
        self.sync = "grads"
        self.cast_dtype = cast_dtype
        self.tied = tied                      # [(param, group, first owner's global rank)] on this rank
        self.param_names = param_names
        self.buffer_refs = list(buffer_refs)   # (original name, owner module, local name)
        self.transport = transport
        self.sig_group = sig_group
        self.order = native_runtime.pipeline_order(schedule, stage, nstages, microbatches, self.V)
        self._init_plans(lag)
        S, SV = nstages, nstages * self.V
        self._vs = [virtual_stage(c, stage, S) for c in range(self.V)]
        self.holds_first = 0 in self._vs
        self.holds_last = (SV - 1) in self._vs
        dev = rt.device()
        # A collective over every group first: each RCCL communicator exists (and has run a
        # collective, which RCCL requires before a batch naming only some of its ranks) before
        # the first point-to-point batch.
        if dist.is_initialized():
            probe = torch.zeros(1, device=dev)
            seen = set()
            extra = [transport.groups["grad"]] if transport is not None else []
            for g in [groups.pp_group, groups.dp_group] + extra:
                if id(g) not in seen:
                    seen.add(id(g))
                    comm.all_reduce(probe, "sum", group=g)
            for _, g, _ in tied:
                comm.all_reduce(probe, "sum", group=g)
            if dev.type == "cuda":
                torch.cuda.synchronize()
        self._sig = _UNSET
        self._in_meta: Dict[int, tuple] = {}    # chunk -> (shape, dtype) of its received activation
        self._out_meta: Dict[int, tuple] = {}   # chunk -> (shape, dtype) of its sent activation
        self._tied_works = []
        self._needs_tied = False
        self.unpack_to_params = False   # a plain torch optimizer reads p.grad (build_pipeline)
        self.last_loss = None
        self.stats = {"steps": 0, "p2p_batches": 0}

    def _init_plans(self, lag: float) -> None:
        """The issue plans this rank can run (:func:`issue_plan` at ``lag`` 0 and at the planned
        transfer time) and how the engine picks one: ``MADNN_PP_PLAN`` = ``auto`` (default: time
        both on the job -- the hardware-queue mapping decides which is faster -- and keep the
        faster), ``0`` (lag 0 only) or ``lag`` (the lagged plan only).  Every plan is deadlock-free
        fully serialised, and every rank switches at the same step, so any mix is safe."""
        import os

        S, M, V = self.nstages, self.M, self.V
        mode = os.environ.get("MADNN_PP_PLAN", "auto")
        lag = plan_lag(lag)
        lags = [0.0]
        if mode != "0" and lag > 0 and any(issue_plan(self.schedule, s, S, M, V) !=
                                           issue_plan(self.schedule, s, S, M, V, lag) for s in range(S)):
            lags = [lag] if mode == "lag" else [0.0, lag]
        self._lags = lags
        self._plans = [issue_plan(self.schedule, self.stage, S, M, V, g) for g in lags]
        self.plan_items = self._plans[0]
        self.plan_lag = lags[0]
        # steps 1 .. 2L run the L plans alternately (step 0 exchanges the shape headers); the plan
        # of a step is a function of the step count alone, so every rank runs the same one
        self._tune = {"t": [0.0] * len(lags), "n": [0] * len(lags), "chosen": 0 if len(lags) == 1 else None}

    def _tune_begin(self, new_sig: bool):
        L, n = len(self._plans), self.stats["steps"]
        if L == 1 or not 1 <= n <= 2 * L:
            return None
        i = (n - 1) % L
        self.plan_items, self.plan_lag = self._plans[i], self._lags[i]
        if torch.cuda.is_available() and rt.device().type == "cuda":
            torch.cuda.synchronize()
        return i, time.perf_counter(), new_sig

    def _tune_end(self, tok) -> None:
        if tok is None:
            return
        i, t0, new_sig = tok
        if torch.cuda.is_available() and rt.device().type == "cuda":
            torch.cuda.synchronize()
        tn = self._tune
        if not new_sig:                      # a step that also exchanged headers is not timed
            tn["t"][i] += time.perf_counter() - t0
            tn["n"][i] += 1
        if self.stats["steps"] != 2 * len(self._plans):
            return
        t = torch.tensor([tt / max(nn_, 1) for tt, nn_ in zip(tn["t"], tn["n"])], dtype=torch.float64)
        if dist.is_initialized() and dist.get_world_size() > 1:
            # the job's time per plan is its slowest rank's; every rank takes the same decision
            dev = rt.device() if dist.get_backend() == "nccl" else torch.device("cpu")
            t = t.to(dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t = t.cpu()
        best = int(torch.argmin(t))
        tn["chosen"] = best
        tn["ms"] = [round(float(x) * 1e3, 3) for x in t]
        self.plan_items, self.plan_lag = self._plans[best], self._lags[best]

    @property
    def is_first(self):
        return self.stage == 0

    @property
    def is_last(self):
        return self.stage == self.nstages - 1

    # ------------------------------------------------------------ training
    def train_step(self, inputs: Optional[torch.Tensor], targets: Optional[torch.Tensor] = None):
        """Forward + backward of every microbatch on this rank; returns the mean loss on the
        rank that holds the last virtual stage (None elsewhere)."""
        self.module.train()
        M, S, SV = self.M, self.nstages, self.nstages * self.V
        if self.holds_first:
            xs = list(inputs.chunk(M))
            if len(xs) != M:
                raise ValueError(f"batch of {inputs.shape[0]} does not split into {M} microbatches")
        if self.holds_last:
            if targets is None:
                raise ValueError("the last pipeline stage needs targets")
            ts = list(targets.chunk(M))
            if len(ts) != M:
                raise ValueError(f"targets of {targets.shape[0]} do not split into {M} microbatches")
        # the header exchange is keyed on the batch signature; ranks without the first / last
        # chunk may pass None, so the pipeline agrees on "new signature" every step (a host-side
        # MAX over the replica's ranks: no device synchronisation)
        ref = inputs if inputs is not None else targets
        sig = (tuple(ref.shape), ref.dtype) if ref is not None else "static"
        new_sig = sig != self._sig
        if self.sig_group is not None and dist.get_world_size(self.sig_group) > 1:
            flag = torch.tensor([1 if new_sig else 0], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.sig_group)
            new_sig = bool(flag.item())
        if self.dp._needs_finalize:
            # gradient accumulation across train_step calls (no optimizer step in between)
            if self.tied:
                # the tied slots already hold the cross-stage SUM; summing them again at the end
                # of this step would count the first step's gradients twice
                raise RuntimeError("pipeline: train_step called again before optimizer.step() with parameters "
                                   "tied across stages; accumulate with more microbatches instead")
            if self.dp.comm_stream is not None:
                # this step's in-place accumulation must follow the previous step's reduction
                torch.cuda.current_stream().wait_stream(self.dp.comm_stream)
        if self._needs_tied:
            self._wait_tied()
        tune = self._tune_begin(new_sig)
        inbox: Dict[tuple, torch.Tensor] = {}     # ("act"|"grad", c, m) -> received tensor
        outbox: Dict[tuple, torch.Tensor] = {}    # ("act"|"grad", c, m) -> tensor to send
        acts_in: Dict[tuple, torch.Tensor] = {}
        acts_out: Dict[tuple, torch.Tensor] = {}
        losses: Dict[tuple, torch.Tensor] = {}
        total = torch.zeros((), device=rt.device(), dtype=torch.float32) if self.holds_last else None
        met_in, met_out = set(), set()
        tp = self.transport
        for item in self.plan_items:
            if item[0] == "X":
                batch = item[1]
                if new_sig:
                    hs, hr = [], []
                    for d, k, c, m, p in batch:
                        if k != "act":
                            continue
                        if d == "send" and c not in met_out:
                            t = outbox[("act", c, m)]
                            self._out_meta[c] = (tuple(t.shape), t.dtype)
                            met_out.add(c)
                            hs.append((t, p))
                        elif d == "recv" and c not in met_in:
                            met_in.add(c)
                            hr.append((c, p))
                    if hs or hr:
                        for (c, _p), meta in zip(hr, tp.exchange_meta(hs, [p for _, p in hr])):
                            self._in_meta[c] = meta
                sends, recvs, keys = [], [], []
                for d, k, c, m, p in batch:
                    if d == "send":
                        sends.append((k, outbox.pop((k, c, m)), p))
                    else:
                        keys.append((k, c, m))
                        recvs.append((k, *(self._in_meta[c] if k == "act" else self._out_meta[c]), p))
                for key, t in zip(keys, tp.exchange_batch(sends, recvs)):
                    inbox[key] = t
                continue
            _, op, c, m = item
            vs = self._vs[c]
            if op == "F":
                if vs == 0:
                    x = _cast_inputs(xs[m], self.cast_dtype, False)
                else:
                    x = inbox.pop(("act", c, m))
                    x.requires_grad_(x.is_floating_point())
                acts_in[(c, m)] = x
                y = self.chunks[c](x)
                if vs == SV - 1:
                    loss = scaled_loss(self.loss_fn, y, ts[m], 1.0 / M)
                    losses[(c, m)] = loss
                    total.add_(loss.detach().float())
                else:
                    acts_out[(c, m)] = y
                    outbox[("act", c, m)] = y
            else:
                ctx = self.dp.no_sync() if m != M - 1 else _null()  # reduce during each chunk's last backward
                with ctx:
                    if vs == SV - 1:
                        losses.pop((c, m)).backward()
                    else:
                        torch.autograd.backward(acts_out.pop((c, m)), grad_tensors=inbox.pop(("grad", c, m)))
                x = acts_in.pop((c, m))
                if vs > 0:
                    outbox[("grad", c, m)] = x.grad if x.grad is not None else torch.zeros_like(x)
        if outbox or inbox:
            raise RuntimeError(f"pipeline plan left messages behind: out {sorted(outbox)} in {sorted(inbox)}")
        self._sig = sig
        self.dp.flush()                      # buckets of params that got no gradient, backward-end event
        self._launch_tied()
        if tp is not None:
            tp.drain()
            self.stats["p2p_batches"] = tp.batches
        self._tune_end(tune)
        self.stats["steps"] += 1
        self.last_loss = total
        if self.unpack_to_params:
            # a plain torch optimizer: p.grad holds the final (reduced, tied-summed) gradients as
            # soon as train_step returns, so anything between it and opt.step() -- gradient
            # clipping, inspection -- sees and changes what the step will apply
            self.finalize_grads()
        return total

    # -------------------------------------------------- tied parameters (N8)
    def _launch_tied(self):
        """Sum the gradients of parameters shared across pipeline ranks (GPT-2's wte/lm_head)
        asynchronously, right after their stage-local DP reduction was issued; the optimizer
        updates the other buckets first and waits for these last (``bucket_order``)."""
        self._tied_works = []
        if not self.tied:
            return
        space = self.dp.space
        cs = self.dp.comm_stream
        for p, group, _src in self.tied:
            bk, off, _ = space.param_info[id(p)]
            buf = space.grad_buffer(bk)[off:off + p.numel()]
            if cs is not None:
                with torch.cuda.stream(cs):
                    if bk.work is not None:
                        bk.work.wait()
                    self._tied_works.append(comm.all_reduce(buf, "sum", group=group, async_op=True))
            else:
                if bk.work is not None:
                    bk.work.wait()
                self._tied_works.append(comm.all_reduce(buf, "sum", group=group, async_op=True))
        self._needs_tied = True

    def _wait_tied(self):
        cs = self.dp.comm_stream
        for w in self._tied_works:
            if w is None:
                continue
            if cs is not None:
                with torch.cuda.stream(cs):
                    w.wait()
            else:
                w.wait()
        if cs is not None and self._tied_works:
            torch.cuda.current_stream().wait_stream(cs)
        self._tied_works = []
        self._needs_tied = False

    # -------------------------------------------------- optimizer protocol
    def finalize_grads(self, wait_tied: bool = True):
        """Idempotent: the stage-local DP reduction, then the cross-stage tied-gradient sum.
        Called by clip_grad_norm_ AND step; the tied sum is applied exactly once per step.
        With a plain torch optimizer (``unpack_to_params``) the final flat gradients are then
        copied into ``p.grad`` -- after the tied sum, so a tied weight's .grad holds both stages'."""
        pending = self.dp._needs_finalize or self._needs_tied
        self.dp.finalize_grads()
        if wait_tied and self._needs_tied:
            self._wait_tied()
        if pending and self.unpack_to_params and not self._needs_tied:
            for bk in self.dp.space.buckets:
                self.dp.space.unpack_grads_to_params(bk)

    def tied_buckets(self) -> set:
        """Buckets holding a tied parameter: the optimizer updates them last, after the others
        (whose gradients are final as soon as the DP reduction is), hiding the tied sum."""
        return {self.dp.space.param_info[id(p)][0].index for p, _, _ in self.tied}

    def norm_reduction(self):
        """(groups to sum squared gradient norms over, params to leave out of this rank's sum):
        pipeline ranks hold disjoint parameters except tied ones, counted on their first owner."""
        skip = [p for p, _g, src in self.tied if src != rt.get_rank()]
        # the pipeline mesh has no tensor-parallel axis (build_pipeline: tp=1); a TP x PP layout
        # would also have to sum over the tp group and skip TP-replicated parameters
        assert self.groups.mesh.tp == 1, "clip_grad_norm_ over a tp x pp mesh is not supported"
        return ([self.groups.pp_group] if self.nstages > 1 else []), skip

    def after_step(self):
        self.dp.after_step()

    def comm_metrics(self) -> dict:
        """DP all-reduce numbers of this stage, P2P bytes, plus the schedule's bubble fraction
        (simulated for the configured schedule; (S-1)/(M+S-1) for GPipe/1F1B)."""
        out = self.dp.comm_metrics()
        out["bubble_fraction"] = pipeline_bubble(self.schedule, self.nstages, self.M, self.V)
        tp = self.transport
        out["p2p_bytes"] = tp.bytes if tp is not None else 0
        out["p2p_batches_per_step"] = (tp.batches / max(self.stats["steps"], 1)) if tp is not None else 0
        out["plan_lags"] = list(self._lags)
        out["plan_lag"] = self.plan_lag
        out["plan_step_ms"] = self._tune.get("ms")
        return out

    # ------------------------------------------------------------ inference
    @torch.no_grad()
    def forward_step(self, inputs: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """Pipelined forward only, microbatch-major then chunk order: each activation travels as
        a header exchange and a data exchange with the next rank (every program a chain along
        the virtual stages, so it completes fully serialised); returns the full output on the
        rank holding the last virtual stage."""
        self.module.eval()
        M, S, SV = self.M, self.nstages, self.nstages * self.V
        xs = list(inputs.chunk(M)) if self.holds_first else [None] * M
        outs = []
        tp = self.transport
        for m in range(M):
            for c in range(self.V):
                vs = self._vs[c]
                if vs == 0:
                    x = _cast_inputs(xs[m], self.cast_dtype, False)
                else:
                    prev = (self.stage - 1) % S
                    shape, dt = tp.exchange_meta([], [prev])[0]
                    x = tp.exchange([], [(shape, dt, prev)])[0]
                y = self.chunks[c](x)
                if vs == SV - 1:
                    outs.append(y)
                else:
                    nxt = (self.stage + 1) % S
                    tp.exchange_meta([(y, nxt)], [])
                    tp.exchange([(y, nxt)], [])
        if tp is not None:
            tp.drain()
        return torch.cat(outs) if outs else None

    def state_dict(self):
        """This rank's parameters under their ORIGINAL model names."""
        out = {}
        for p in self.module.parameters():
            name = self.param_names.get(id(p))
            if name is not None:
                out[name] = p
        return out

    def named_buffers(self):
        for name, owner, local in self.buffer_refs:
            yield name, owner.get_buffer(local)


_BUBBLE_CACHE: Dict[tuple, float] = {}
_TRANSPORT_CACHE: Dict[tuple, float] = {}


def transport_time(schedule: str, nstages: int, nmicro: int, nchunks: int, chunk_s: float, p2p_s: float) -> float:
    """Seconds of one pipelined step of ``nmicro`` microbatches when one chunk's forward +
    backward of one microbatch takes ``chunk_s`` (split 1 : 2) and one activation / gradient
    transfer ``p2p_s``: the makespan of :func:`simulate_transport` on the engine's transport
    (independent queues), so the planner prices exactly the communication this engine exposes --
    the better of its two issue plans (``lag`` 0 and the transfer time), as the engine keeps the
    one that measured faster.  Cached on the transfer / compute ratio (2 significant digits)."""
    if nstages <= 1 or chunk_s <= 0:
        return nmicro * nchunks * max(chunk_s, 0.0)
    ratio = float(f"{p2p_s / chunk_s:.2g}") if p2p_s > 0 else 0.0
    key = (schedule, nstages, nmicro, nchunks, ratio)
    if key not in _TRANSPORT_CACHE:
        t = [simulate_transport(schedule, nstages, nmicro, nchunks, "split", None, t_fwd=1.0, t_bwd=2.0,
                                t_p2p=3.0 * ratio, lag=lag)["makespan"] / 3.0
             for lag in sorted({0.0, plan_lag(3.0 * ratio)})]
        _TRANSPORT_CACHE[key] = min(t)
    return _TRANSPORT_CACHE[key] * chunk_s


def pipeline_bubble(schedule: str, nstages: int, nmicro: int, nchunks: int = 1) -> float:
    """Idle fraction of a schedule (backward = 2x forward), from :func:`simulate_schedule`."""
    key = (schedule, nstages, nmicro, nchunks)
    if key not in _BUBBLE_CACHE:
        if nstages <= 1:
            _BUBBLE_CACHE[key] = 0.0
        else:
            _BUBBLE_CACHE[key] = simulate_schedule(schedule, nstages, nmicro, nchunks)["bubble"]
    return _BUBBLE_CACHE[key]


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


_UNSET = object()


def _chunk_layer_ranges(plan, stage: int, nstages: int, V: int):
    """(lo, hi) spine-layer ranges of this rank's chunks: chunk c = virtual stage c*S + stage."""
    return [(plan.bounds[virtual_stage(c, stage, nstages)], plan.bounds[virtual_stage(c, stage, nstages) + 1])
            for c in range(V)]


def build_pipeline(model: nn.Module, optimizer, cfg: Config, plan, loss_fn: Optional[Callable] = None):
    """Cut ``model`` along ``plan`` and return ``(PipelineEngine, stage_optimizer)`` for this rank."""
    from ..api import _is_fused, build_space, prepare_model

    rt.init(timeout_s=cfg.timeout_s)
    world = rt.get_world_size()
    S = plan.pp
    V = max(int(getattr(plan, "virtual", 1) or 1), 1)
    schedule = getattr(plan, "schedule", None) or cfg.schedule
    if V > 1:
        schedule = "interleaved"
    elif schedule in ("interleaved", "auto", "none"):
        schedule = "1f1b"
    if len(plan.bounds) != S * V + 1:
        raise ValueError(f"plan has {len(plan.bounds) - 1} pipeline chunks, expected {S} x {V}")
    mesh = rt.Mesh(dp=plan.dp, pp=S, tp=1)
    if mesh.size != world:
        raise ValueError(f"plan {plan.dp}x{S} does not match world size {world}")
    groups = rt.ProcessGroups(mesh)
    # the gradient communicator of every pipeline replica (same ranks as its pipeline group)
    grad_groups = []
    # a host-side (gloo) group per replica for the per-step input-signature agreement: ranks
    # without the first / last chunk may pass None and cannot see a shape change themselves
    sig_groups = []
    if S > 1:
        gloo = dist.is_initialized() and dist.get_backend() == "gloo"
        for d in range(plan.dp):
            ranks = [mesh.rank_of(d, s, 0) for s in range(S)]
            grad_groups.append(dist.new_group(ranks) if dist.is_initialized() else None)
            sig_groups.append(None if not dist.is_initialized() else
                              grad_groups[-1] if gloo else dist.new_group(ranks, backend="gloo"))
    stage = groups.pp_idx
    ranges = _chunk_layer_ranges(plan, stage, S, V)
    all_layers = plan.spine.layers

    # tied parameters, from ORIGINAL parameter identities (before this rank materialises its
    # chunks, which re-creates the local tensors): which pipeline ranks hold each shared one
    pid_name = {}
    for n, p in model.named_parameters(remove_duplicate=False):
        pid_name.setdefault(id(p), n)
    owners: Dict[str, List[int]] = {}
    for vs in range(S * V):
        for layer in all_layers[plan.bounds[vs]:plan.bounds[vs + 1]]:
            for p in layer.parameters():
                name = pid_name.get(id(p))
                if name is None:
                    continue
                lst = owners.setdefault(name, [])
                if vs % S not in lst:
                    lst.append(vs % S)
    tied_sets = [(n, sorted(sts)) for n, sts in owners.items() if len(sts) > 1]

    layers_per_chunk = [all_layers[lo:hi] for lo, hi in ranges]
    flat_layers = [l for ls in layers_per_chunk for l in ls]
    pmap, bmap = original_names(model, flat_layers)
    chunks = [StageModule(ls, plan.checkpoint[lo:hi]) for ls, (lo, hi) in zip(layers_per_chunk, ranges)]
    stage_mod = PipelineStage(chunks)
    dev = rt.device()
    init_fn = getattr(model, "init_weights", None)
    materialize_(stage_mod, dev, init_fn)
    stage_mod.to(dev)
    loss_fn = loss_fn or getattr(model, "loss_fn", None)
    if loss_fn is None:
        from ..models.hf import hf_loss_fn

        loss_fn = hf_loss_fn(model)
    if loss_fn is None:
        raise ValueError("pipeline parallelism needs loss_fn= (or model.loss_fn)")

    names, buffer_refs = stage_names(flat_layers, pmap, bmap)
    by_name = {n: p for p in stage_mod.parameters() for n in [names.get(id(p))] if n is not None}
    tied_local = []
    for name, sts in tied_sets:  # every rank creates every group, same order
        for d in range(plan.dp):
            ranks = [mesh.rank_of(d, s, 0) for s in sts]
            grp = dist.new_group(ranks) if dist.is_initialized() else None
            if rt.get_rank() in ranks:
                tied_local.append((by_name[name], grp, ranks[0]))

    # activations travel on the replica's pipeline group, gradients on a second group over the
    # same ranks (issue_plan / P2PTransport); every rank creates every replica's group, in order
    transport = P2PTransport(groups.pp_group, grad_groups[groups.dp_idx], groups.pp_ranks, dev) if S > 1 else None

    dtype, dtype_of, cl = prepare_model(stage_mod, cfg, dev)
    stage_params = [p for p in stage_mod.parameters() if p.requires_grad]
    if optimizer is not None:
        optimizer = restrict_optimizer(optimizer, stage_params)
    space = build_space(stage_mod, optimizer, cfg, dev, dtype_of, cl)
    # identical copies of tied params: take the first owner stage's values
    with torch.no_grad():
        for p, grp, src in tied_local:
            t = space.master_view(p).contiguous()
            comm.broadcast(t, src=src, group=grp)
            space.master_view(p).copy_(t)
        space.sync_model_from_master()
    dp_engine = DataParallel(stage_mod, space, group=groups.dp_group, src_rank=groups.dp_ranks[0], sync="grads",
                             overlap=cfg.overlap, cast_dtype=dtype, channels_last=cl, unpack_grads=False,
                             broadcast_buffers=cfg.broadcast_buffers, find_unused=True, sync_comm=cfg.sync_comm,
                             rebuild_buckets=cfg.rebuild_buckets and optimizer is not None)
    engine = PipelineEngine(stage_mod, stage=stage, nstages=S, groups=groups, microbatches=plan.microbatches,
                            schedule=schedule, loss_fn=loss_fn, dp_engine=dp_engine, cast_dtype=dtype,
                            tied=tied_local, param_names=names, buffer_refs=buffer_refs, transport=transport,
                            lag=_planned_lag(plan),
                            sig_group=sig_groups[groups.dp_idx] if sig_groups else None)
    engine.plan = plan
    if optimizer is not None and _is_fused(optimizer):
        optimizer.bind(space)
        optimizer.grad_source = engine
        optimizer.nonfinite = cfg.nonfinite
        dp_engine.optimizer = optimizer
    elif optimizer is not None:
        # a plain torch optimizer (as the DP path accepts, api._distribute_dp): it steps the stage's
        # own parameters from p.grad; the engine fills p.grad before the step and re-syncs its flat
        # master copy after it
        engine.unpack_to_params = True
        optimizer.register_step_pre_hook(lambda *a, **k: engine.finalize_grads())

        def _after_plain(*a, **k):
            space.sync_master_from_model()
            engine.after_step()

        optimizer.register_step_post_hook(_after_plain)
    get_logger().info("madnn pp: rank %d/%d chunks %s dp=%d microbatches=%d schedule=%s tied=%d", stage, S,
                      ranges, plan.dp, plan.microbatches, schedule, len(tied_local))
    return engine, optimizer
