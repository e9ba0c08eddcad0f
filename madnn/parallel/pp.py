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
* communication is derived from that order over one-directional FIFO
  channels, each its own process group (own RCCL communicator and stream):
  activations r -> r+1 (ring edge S-1 -> 0 between chunks), gradients back.
  Every receive of a step is posted up front and consumed with a stream wait,
  sends are never waited on before the step ends, so the xGMI transfers run
  underneath compute (``simulate_schedule`` proves each channel's receive
  order equals its send order, which is what makes that legal);
* gradients of each rank are reduced over its DP group by the bucketed
  ``DataParallel`` reducer during each chunk's LAST microbatch backward
  (``no_sync`` before) on links disjoint from the PP hops;
* parameters shared by two ranks (GPT-2's tied ``wte``/``lm_head``) have
  their gradients summed between the owners asynchronously right after the
  last backward; the optimizer updates every other bucket first.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist
from torch import nn
from torch.utils.checkpoint import checkpoint

from .. import comm
from .. import runtime as rt
from ..config import Config
from ..ops import native_runtime
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
    return type(opt)(groups, **opt.defaults)


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
    return {"makespan": makespan, "bubble": 1.0 - max(busy) / makespan, "peak_inflight": peak}


# ----------------------------------------------------------------------------
# channel layout (shared by build_pipeline and the transport simulation)
# ----------------------------------------------------------------------------
def p2p_channel_specs(nstages: int, nchunks: int = 1) -> List[tuple]:
    """The one-directional channels of one pipeline replica, in creation order, as
    ``(name at the sender, name at the receiver, sender stage, receiver stage)``: activations
    on every edge s -> s+1, gradients on every edge s+1 -> s, and with V > 1 the ring edge
    (activations S-1 -> 0 between chunks, their gradients 0 -> S-1)."""
    S = nstages
    specs = [("act_out", "act_in", e, e + 1) for e in range(S - 1)]
    specs += [("grad_out", "grad_in", e + 1, e) for e in range(S - 1)]
    if nchunks > 1:
        specs += [("act_out_wrap", "act_in_wrap", S - 1, 0), ("grad_out_wrap", "grad_in_wrap", 0, S - 1)]
    return specs


def p2p_group_layout(nstages: int, nchunks: int, dp: int, rank_of: Callable[[int, int], int],
                     layout: str = "pairwise") -> List[tuple]:
    """The process groups that carry the pipeline channels, in creation order (every rank must
    call ``new_group`` for all of them, members or not), as ``(ranks, [(replica, spec), ...])``.

    ``pairwise`` (the engine's layout): ONE 2-rank group per channel, i.e. per (edge,
    direction, replica).  On RCCL with eager initialisation an unbatched send/recv is executed
    like a collective, in issue order with every other op on its communicator; a group with a
    single sender and a single receiver is therefore a true FIFO whose pre-posted receives can
    never block a send of the same rank.  ``shared`` (round-2 layout, kept only so the transport
    tests can show that it deadlocks): one S-rank group per channel kind and replica, where an
    interior rank's sends queue behind its own pre-posted receives."""
    specs = p2p_channel_specs(nstages, nchunks)
    out = []
    if layout == "pairwise":
        for d in range(dp):
            for sp in specs:
                out.append(((rank_of(d, sp[2]), rank_of(d, sp[3])), [(d, sp)]))
    elif layout == "shared":
        kinds = ["act", "grad"] + (["act_wrap", "grad_wrap"] if nchunks > 1 else [])
        for kind in kinds:
            for d in range(dp):
                carried = [(d, sp) for sp in specs if sp[0].replace("_out", "") == kind]
                out.append((tuple(rank_of(d, s) for s in range(nstages)), carried))
    else:
        raise ValueError(f"unknown pipeline channel layout {layout!r}")
    return out


def recv_plan(order, vstages: List[int], nvirtual: int) -> List[tuple]:
    """Every receive one pipeline rank makes in a step, in issue order: ``("act", c, m)`` before
    the forward of virtual stage c*S+rank (unless it is the first), ``("grad", c, m)`` before the
    backward of every virtual stage but the last.  The engine pre-posts exactly this list."""
    out = []
    for op, c, m in order:
        vs = vstages[c]
        if op == "F" and vs > 0:
            out.append(("act", c, m))
        elif op == "B" and vs < nvirtual - 1:
            out.append(("grad", c, m))
    return out


def _chan_names(stage: int, nstages: int):
    """This rank's channel names: (act in, act out, grad in, grad out)."""
    return ("act_in" if stage > 0 else "act_in_wrap", "act_out" if stage < nstages - 1 else "act_out_wrap",
            "grad_in" if stage < nstages - 1 else "grad_in_wrap", "grad_out" if stage > 0 else "grad_out_wrap")


def simulate_transport(kind: str, nstages: int, nmicro: int, nchunks: int = 1, layout: str = "pairwise",
                       prepost: bool = True, t_fwd: float = 1.0, t_bwd: float = 2.0, t_p2p: float = 0.0) -> dict:
    """Replay one training step of every pipeline rank against the COMMUNICATORS
    :func:`p2p_group_layout` builds, with RCCL's eager-initialisation semantics.

    Model: each rank has a compute stream and one stream per communicator it belongs to; all of
    a rank's operations on one communicator execute in issue order (unbatched P2P is serialised
    like a collective).  The host issues, in program order, the receives of :func:`recv_plan`
    (all up front when ``prepost``; otherwise each right before its consumer, preceded by the
    shape header that the first step of a new input signature exchanges with a host-blocking
    receive), every forward/backward on the compute stream (waiting on its receive), and each
    send on its channel's communicator right after its producer.  A send completes only
    together with the matching receive at the head of the peer's stream (rendezvous, the
    conservative reading of RCCL's P2P protocol).  Raises RuntimeError on a deadlock or when a
    receive would be matched with a message meant for another receive; otherwise returns
    ``{"makespan", "bubble", "communicators"}``."""
    S, M, V = nstages, nmicro, nchunks
    SV = S * V
    groups = p2p_group_layout(S, V, 1, lambda d, s: s, layout)
    comm_of: Dict[tuple, int] = {}
    for gi, (_ranks, carried) in enumerate(groups):
        for _d, (n_src, n_dst, a, b) in carried:
            comm_of[(a, n_src)] = gi
            comm_of[(b, n_dst)] = gi
    ops: List[dict] = []           # every op: kind C/S/R, rank, stream, deps, payload

    def new(kind_, rank, stream, **kw):
        ops.append(dict(kind=kind_, rank=rank, stream=stream, done=None, **kw))
        return len(ops) - 1

    programs = []                  # per rank: list of ("issue", op id) / ("hostwait", op id)
    for s in range(S):
        order = native_runtime.pipeline_order(kind, s, S, M, V)
        vst = [virtual_stage(c, s, S) for c in range(V)]
        a_in, a_out, g_in, g_out = _chan_names(s, S)
        prog = []
        recv_id: Dict[tuple, int] = {}
        met_in, met_out = set(), set()

        def post(key, s=s, a_in=a_in, g_in=g_in, vst=vst, recv_id=recv_id, prog=prog):
            k, c, m = key
            name = a_in if k == "act" else g_in
            peer = (s - 1) % S if k == "act" else (s + 1) % S
            msg = (k, vst[c], m)
            recv_id[key] = new("R", s, ("comm", comm_of[(s, name)]), peer=peer, msg=msg)
            prog.append(("issue", recv_id[key]))

        if prepost:
            for key in recv_plan(order, vst, SV):
                post(key)
        for op, c, m in order:
            vs = vst[c]
            dep = None
            if op == "F" and vs > 0 or op == "B" and vs < SV - 1:
                key = ("act" if op == "F" else "grad", c, m)
                if not prepost:
                    if op == "F" and c not in met_in:   # shape header, host-blocking
                        met_in.add(c)
                        h = new("R", s, ("comm", comm_of[(s, a_in)]), peer=(s - 1) % S, msg=("hdr", vs, c))
                        prog.append(("issue", h))
                        prog.append(("hostwait", h))
                    post(key)
                dep = recv_id[key]
            cid = new("C", s, ("compute",), dep=dep, dur=t_fwd if op == "F" else t_bwd)
            prog.append(("issue", cid))
            if op == "F" and vs < SV - 1:
                if not prepost and c not in met_out:
                    met_out.add(c)
                    prog.append(("issue", new("S", s, ("comm", comm_of[(s, a_out)]), peer=(s + 1) % S,
                                              msg=("hdr", vs + 1, (vs + 1) // S), dep=cid)))
                prog.append(("issue", new("S", s, ("comm", comm_of[(s, a_out)]), peer=(s + 1) % S,
                                          msg=("act", vs + 1, m), dep=cid)))
            elif op == "B" and vs > 0:
                prog.append(("issue", new("S", s, ("comm", comm_of[(s, g_out)]), peer=(s - 1) % S,
                                          msg=("grad", vs - 1, m), dep=cid)))
        programs.append(prog)

    pc = [0] * S
    queues: Dict[tuple, list] = {}   # (rank, stream) -> op ids in issue order (FIFO)
    free: Dict[tuple, float] = {}
    busy = [0.0] * S
    remaining = len(ops)

    def head(rank, stream):
        q = queues.get((rank, stream))
        return q[0] if q else None

    while remaining:
        progressed = False
        for s in range(S):               # the host issues until it reaches an unfinished wait
            prog = programs[s]
            while pc[s] < len(prog):
                what, oid = prog[pc[s]]
                if what == "hostwait":
                    if ops[oid]["done"] is None:
                        break
                else:
                    queues.setdefault((s, ops[oid]["stream"]), []).append(oid)
                pc[s] += 1
                progressed = True
        for (s, stream), q in list(queues.items()):
            while q:
                o = ops[q[0]]
                if o["kind"] == "C":
                    if o["dep"] is not None and ops[o["dep"]]["done"] is None:
                        break
                    start = max(free.get((s, stream), 0.0), ops[o["dep"]]["done"] if o["dep"] is not None else 0.0)
                    o["done"] = start + o["dur"]
                    busy[s] += o["dur"]
                elif o["kind"] == "S":
                    if ops[o["dep"]]["done"] is None:
                        break
                    ph = head(o["peer"], stream)
                    if ph is None or ops[ph]["kind"] != "R" or ops[ph]["peer"] != s:
                        break
                    r = ops[ph]
                    if r["msg"] != o["msg"]:
                        raise RuntimeError(f"transport {layout} {kind} S={S} M={M} V={V}: rank {o['peer']} "
                                           f"receives {o['msg']} where it expects {r['msg']}")
                    start = max(free.get((s, stream), 0.0), free.get((o["peer"], stream), 0.0),
                                ops[o["dep"]]["done"])
                    o["done"] = r["done"] = start + t_p2p
                    free[(o["peer"], stream)] = r["done"]
                    queues[(o["peer"], stream)].pop(0)
                    remaining -= 1
                else:
                    break                # a receive completes with its matching send
                free[(s, stream)] = o["done"]
                q.pop(0)
                remaining -= 1
                progressed = True
        if not progressed:
            stuck = {}
            for (s, stream), q in queues.items():
                if q:
                    o = ops[q[0]]
                    stuck.setdefault(s, []).append((stream, o["kind"], o.get("msg")))
            raise RuntimeError(f"pipeline transport {layout} {kind} S={S} M={M} V={V} deadlocks; "
                               f"stream heads: {stuck}")
    makespan = max(o["done"] for o in ops)
    return {"makespan": makespan, "bubble": 1.0 - max(busy) / makespan if makespan else 0.0,
            "communicators": len(groups)}


# ----------------------------------------------------------------------------
# transport
# ----------------------------------------------------------------------------
class _SerialWork:
    """Completion handle of an op run by :class:`_SerialComm` (wait() raises on a timeout)."""

    __slots__ = ("event", "error", "timeout")

    def __init__(self, timeout):
        import threading

        self.event = threading.Event()
        self.error = None
        self.timeout = timeout

    def wait(self):
        if not self.event.wait(self.timeout):
            raise RuntimeError(f"emulated RCCL P2P: operation not complete after {self.timeout:.0f} s "
                               "(the communicator's FIFO is blocked: transport deadlock)")
        if self.error is not None:
            raise self.error
        return True


class _SerialComm:
    """CPU test double of an eagerly initialised RCCL communicator: every point-to-point
    operation on the group runs to completion, one at a time, in issue order, on one worker
    thread (``MADNN_EMULATE_RCCL_P2P=1`` on gloo).  Gloo alone completes sends and receives of
    different peers independently, which hides the serialisation RCCL imposes."""

    _by_group: Dict[int, "_SerialComm"] = {}

    def __init__(self, timeout):
        import queue
        import threading

        self.q = queue.Queue()
        self.timeout = timeout
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    @classmethod
    def of(cls, group, timeout):
        c = cls._by_group.get(id(group))
        if c is None:
            c = cls._by_group[id(group)] = cls(timeout)
        return c

    def _run(self):
        while True:
            fn, work = self.q.get()
            try:
                fn().wait()
            except Exception as e:  # noqa: BLE001
                work.error = e
            work.event.set()

    def submit(self, fn) -> _SerialWork:
        w = _SerialWork(self.timeout)
        self.q.put((fn, w))
        return w


def _emulated_p2p_timeout() -> Optional[float]:
    import os

    v = os.environ.get("MADNN_EMULATE_RCCL_P2P", "")
    if v in ("", "0"):
        return None
    return float(os.environ.get("MADNN_EMULATE_RCCL_P2P_TIMEOUT", "60"))
class _Pending:
    """A posted receive; ``get()`` orders the consumer after it (RCCL: a stream wait, no
    host block) and returns the tensor on the compute device."""

    __slots__ = ("work", "buf", "device", "staged")

    def __init__(self, work, buf, device, staged):
        self.work, self.buf, self.device, self.staged = work, buf, device, staged

    def get(self) -> torch.Tensor:
        self.work.wait()
        return self.buf.to(self.device, non_blocking=False) if self.staged else self.buf


class Channel:
    """One-directional point-to-point FIFO between two pipeline ranks.

    Its process group has exactly two ranks, the sender and the receiver
    (:func:`p2p_group_layout`), so its RCCL communicator -- which executes unbatched
    send/recv in issue order on its own HIP stream -- only ever carries messages one way and
    in one order: receives can be posted ahead of time (the transfer runs as soon as the
    peer's send is enqueued, overlapping this rank's compute) and sends are never waited on
    before the end of the step.  On a gloo group HIP tensors are staged through host memory
    (tests run several ranks on one GPU that way; RCCL refuses that); with
    ``MADNN_EMULATE_RCCL_P2P=1`` gloo ops run through :class:`_SerialComm`, which imposes
    RCCL's per-communicator serialisation on the CPU tests."""

    def __init__(self, group, src: int, dst: int, device, name: str = ""):
        self.group, self.src, self.dst, self.name = group, src, dst, name
        self.device = torch.device(device)
        backend = dist.get_backend(group) if dist.is_initialized() else "gloo"
        self.staged = backend == "gloo" and self.device.type == "cuda"
        self.buf_device = torch.device("cpu") if self.staged else self.device
        t = _emulated_p2p_timeout() if backend == "gloo" else None
        self.serial = _SerialComm.of(group, t) if t is not None else None
        self._sends = []
        self.bytes = 0
        self.messages = 0

    def _isend(self, t):
        if self.serial is not None:
            return self.serial.submit(lambda: dist.isend(t, self.dst, group=self.group))
        return dist.isend(t, self.dst, group=self.group)

    def _irecv(self, buf):
        if self.serial is not None:
            return self.serial.submit(lambda: dist.irecv(buf, self.src, group=self.group))
        return dist.irecv(buf, self.src, group=self.group)

    def send(self, t: torch.Tensor) -> None:
        t = t.detach().contiguous()
        if self.staged:
            t = t.cpu()
        comm._record("send", self.group, t)
        self._sends.append((self._isend(t), t))
        self.bytes += t.numel() * t.element_size()
        self.messages += 1

    def post_recv(self, shape, dtype) -> _Pending:
        buf = torch.empty(shape, dtype=dtype, device=self.buf_device)
        comm._record("recv", self.group, buf)
        return _Pending(self._irecv(buf), buf, self.device, self.staged)

    def send_meta(self, t: torch.Tensor) -> None:
        hdr = torch.zeros(10, dtype=torch.int64)
        hdr[0] = t.dim()
        hdr[1] = _DT_CODE[t.dtype]
        hdr[2:2 + t.dim()] = torch.tensor(t.shape, dtype=torch.int64)
        self.send(hdr.to(self.buf_device))

    def recv_meta(self):
        h = self.post_recv((10,), torch.int64).get().tolist()
        return tuple(int(v) for v in h[2:2 + h[0]]), _CODE_DT[h[1]]

    def drain(self) -> None:
        """Wait for (RCCL: order the current stream after) every send of this step."""
        for w, _ in self._sends:
            w.wait()
        self._sends.clear()


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
    chunks per rank); all communication is derived from it: the activation input of every
    non-first virtual stage arrives on the ``act`` channel from the previous rank (the ring
    edge S-1 -> 0 between chunks), gradients flow back on the ``grad`` channels.  In steady
    state every receive of the step is posted up front (shapes are known from the first step
    of an input signature, which exchanges headers just in time), so each transfer overlaps
    the compute that precedes its consumer; sends are fire-and-forget until the step ends."""

    def __init__(self, stage_module: PipelineStage, *, stage: int, nstages: int, groups: rt.ProcessGroups,
                 microbatches: int, schedule: str, loss_fn: Callable, dp_engine: DataParallel,
                 cast_dtype, tied: List[tuple], param_names: Dict[int, str], buffer_refs=(),
                 channels: Optional[Dict[str, Channel]] = None, p2p_groups=()):
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
        self.channels = channels or {}
        self.order = native_runtime.pipeline_order(schedule, stage, nstages, microbatches, self.V)
        S, SV = nstages, nstages * self.V
        self._vs = [virtual_stage(c, stage, S) for c in range(self.V)]
        self.holds_first = 0 in self._vs
        self.holds_last = (SV - 1) in self._vs
        dev = rt.device()
        # A collective over every group first: each RCCL communicator exists before its first
        # point-to-point operation.
        if dist.is_initialized():
            probe = torch.zeros(1, device=dev)
            seen = set()
            for g in [groups.pp_group, groups.dp_group] + list(p2p_groups):
                if id(g) not in seen:
                    seen.add(id(g))
                    comm.all_reduce(probe, "sum", group=g)
            for _, g, _ in tied:
                comm.all_reduce(probe, "sum", group=g)
            self._warm_channels()
        self._sig = _UNSET
        self._in_meta: Dict[int, tuple] = {}    # chunk -> (shape, dtype) of its received activation
        self._out_meta: Dict[int, tuple] = {}   # chunk -> (shape, dtype) of its sent activation
        self._tied_works = []
        self._needs_tied = False
        self.last_loss = None
        self.stats = {"steps": 0, "prefetched_recvs": 0}

    @property
    def is_first(self):
        return self.stage == 0

    @property
    def is_last(self):
        return self.stage == self.nstages - 1

    # ------------------------------------------------------------ channels
    def _warm_channels(self):
        """Create every channel's point-to-point communicator before the first step.

        RCCL builds a two-rank communicator on a pair's first send/recv and that build is a
        blocking rendezvous of the two ranks.  Doing it lazily inside the schedule would turn
        the first message of every channel into a synchronous handshake (the schedule is only
        proven deadlock-free for non-blocking sends); here every rank walks its channels in
        the global group-creation order (then edge index inside a group), so the handshakes
        form a chain that always completes."""
        ranked = sorted(self.channels, key=lambda n: getattr(self.channels[n], "warm_key", (0, 0)))
        for name in ranked:
            ch = self.channels[name]
            t = torch.zeros(1, device=ch.buf_device)
            if name.endswith("_out") or name.endswith("_out_wrap"):
                dist.isend(t, ch.dst, group=ch.group).wait()
            else:
                dist.irecv(t, ch.src, group=ch.group).wait()
        if self.channels and torch.cuda.is_available() and rt.device().type == "cuda":
            torch.cuda.synchronize()

    def _act_in(self, c: int) -> Channel:
        return self.channels["act_in" if self.stage > 0 else "act_in_wrap"]

    def _act_out(self, c: int) -> Channel:
        return self.channels["act_out" if self.stage < self.nstages - 1 else "act_out_wrap"]

    def _grad_in(self, c: int) -> Channel:
        return self.channels["grad_in" if self.stage < self.nstages - 1 else "grad_in_wrap"]

    def _grad_out(self, c: int) -> Channel:
        return self.channels["grad_out" if self.stage > 0 else "grad_out_wrap"]

    def _prepost(self):
        """Post every receive of the step (:func:`recv_plan`, the order
        :func:`simulate_transport` proves deadlock-free on the channel groups)."""
        q = {}
        for key in recv_plan(self.order, self._vs, self.nstages * self.V):
            k, c, _m = key
            if k == "act":
                q[key] = self._act_in(c).post_recv(*self._in_meta[c])
            else:
                q[key] = self._grad_in(c).post_recv(*self._out_meta[c])
        self.stats["prefetched_recvs"] += len(q)
        return q

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
        # every rank of a pipeline must see the same batch SHAPE each step (ranks without the
        # first/last chunk may pass None): the header exchange is keyed on it
        ref = inputs if inputs is not None else targets
        sig = (tuple(ref.shape), ref.dtype) if ref is not None else "static"
        new_sig = sig != self._sig
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
        pend = {} if new_sig else self._prepost()
        acts_in: Dict[tuple, torch.Tensor] = {}
        acts_out: Dict[tuple, torch.Tensor] = {}
        losses: Dict[tuple, torch.Tensor] = {}
        total = torch.zeros((), device=rt.device(), dtype=torch.float32) if self.holds_last else None
        met_in, met_out = set(), set()
        for op, c, m in self.order:
            vs = self._vs[c]
            if op == "F":
                if vs == 0:
                    x = _cast_inputs(xs[m], self.cast_dtype, False)
                else:
                    if new_sig:
                        ch = self._act_in(c)
                        if c not in met_in:
                            self._in_meta[c] = ch.recv_meta()
                            met_in.add(c)
                        x = ch.post_recv(*self._in_meta[c]).get()
                    else:
                        x = pend.pop(("act", c, m)).get()
                    x.requires_grad_(x.is_floating_point())
                acts_in[(c, m)] = x
                y = self.chunks[c](x)
                if vs == SV - 1:
                    loss = self.loss_fn(y, ts[m]) / M
                    losses[(c, m)] = loss
                    total.add_(loss.detach().float())
                else:
                    acts_out[(c, m)] = y
                    ch = self._act_out(c)
                    if new_sig and c not in met_out:
                        self._out_meta[c] = (tuple(y.shape), y.dtype)
                        ch.send_meta(y)
                        met_out.add(c)
                    ch.send(y)
            else:
                ctx = self.dp.no_sync() if m != M - 1 else _null()  # reduce during each chunk's last backward
                with ctx:
                    if vs == SV - 1:
                        losses.pop((c, m)).backward()
                    else:
                        g = (self._grad_in(c).post_recv(*self._out_meta[c]) if new_sig
                             else pend.pop(("grad", c, m))).get()
                        torch.autograd.backward(acts_out.pop((c, m)), grad_tensors=g)
                x = acts_in.pop((c, m))
                if vs > 0:
                    self._grad_out(c).send(x.grad if x.grad is not None else torch.zeros_like(x))
        self._sig = sig
        self.dp.flush()                      # buckets of params that got no gradient, backward-end event
        self._launch_tied()
        for ch in self.channels.values():
            ch.drain()
        self.stats["steps"] += 1
        self.last_loss = total
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
        Called by clip_grad_norm_ AND step; the tied sum is applied exactly once per step."""
        self.dp.finalize_grads()
        if wait_tied and self._needs_tied:
            self._wait_tied()

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
        out["p2p_bytes"] = sum(ch.bytes for ch in self.channels.values())
        return out

    # ------------------------------------------------------------ inference
    @torch.no_grad()
    def forward_step(self, inputs: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """Pipelined forward only, microbatch-major then chunk order (every channel FIFO);
        returns the full output on the rank holding the last virtual stage."""
        self.module.eval()
        M, SV = self.M, self.nstages * self.V
        xs = list(inputs.chunk(M)) if self.holds_first else [None] * M
        outs = []
        for m in range(M):
            for c in range(self.V):
                vs = self._vs[c]
                if vs == 0:
                    x = _cast_inputs(xs[m], self.cast_dtype, False)
                else:
                    ch = self._act_in(c)
                    shape, dt = ch.recv_meta()
                    x = ch.post_recv(shape, dt).get()
                y = self.chunks[c](x)
                if vs == SV - 1:
                    outs.append(y)
                else:
                    ch = self._act_out(c)
                    ch.send_meta(y)
                    ch.send(y)
        for ch in self.channels.values():
            ch.drain()
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

    # one-directional FIFO channels, one 2-rank process group each (p2p_group_layout); every
    # rank creates every group in the same order
    import os

    layout = os.environ.get("MADNN_PP_P2P_LAYOUT", "pairwise")
    channels: Dict[str, Channel] = {}
    p2p_groups = []  # every channel group this rank belongs to (also those it sends nothing on)
    me = rt.get_rank()
    for gidx, (ranks, carried) in enumerate(p2p_group_layout(S, V, plan.dp, lambda d, s: mesh.rank_of(d, s, 0),
                                                             layout)):
        grp = dist.new_group(list(ranks)) if dist.is_initialized() else None
        if me not in ranks:
            continue
        p2p_groups.append(grp)
        for d, (n_src, n_dst, a, b) in carried:
            src, dst = mesh.rank_of(d, a, 0), mesh.rank_of(d, b, 0)
            for name, mine in ((n_src, src), (n_dst, dst)):
                if mine == me:
                    ch = Channel(grp, src, dst, dev, name)
                    ch.warm_key = (gidx, min(a, b))
                    channels[name] = ch

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
                            tied=tied_local, param_names=names, buffer_refs=buffer_refs, channels=channels,
                            p2p_groups=p2p_groups)
    engine.plan = plan
    if optimizer is not None:
        if not _is_fused(optimizer):
            raise TypeError("pipeline engine needs a madnn fused optimizer (FusedSGD / FusedAdam)")
        optimizer.bind(space)
        optimizer.grad_source = engine
        optimizer.nonfinite = cfg.nonfinite
        dp_engine.optimizer = optimizer
    get_logger().info("madnn pp: rank %d/%d chunks %s dp=%d microbatches=%d schedule=%s tied=%d", stage, S,
                      ranges, plan.dp, plan.microbatches, schedule, len(tied_local))
    return engine, optimizer
