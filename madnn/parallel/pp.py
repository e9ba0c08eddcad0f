"""Pipeline-parallel engine (GPipe / 1F1B) and hybrid DP x PP over RCCL.

Not in the reference ("Pipeline parallel — No"); BASELINE
configs 3 and 4 require it.  Design for one MI355X node:

* one process per GPU; rank -> (dp, pp) coordinates from ``runtime.Mesh``;
  the planner's stage boundaries cut the traced spine into per-rank stage
  modules (layers on the META device are materialised only on their own
  rank, so an 8B model never exists whole in host memory);
* the per-stage instruction list — forward/backward AND its send/recv steps —
  comes from the C++ scheduler (``madnn_pipeline_program``); steady-state
  1F1B pairs (send activation / receive gradient) are issued as ONE
  ``batch_isend_irecv`` group so adjacent stages never both block in a send;
* activations travel as bf16 over the xGMI link between adjacent stages
  (every pair of GPUs is one hop on the MI355X mesh); shapes are negotiated
  once per input signature;
* gradients of each stage are reduced over its DP group by the bucketed
  ``DataParallel`` reducer, only during the LAST microbatch's backward
  (``no_sync`` before), so the all-reduce overlaps that backward and travels
  on links disjoint from the PP hops;
* parameters shared by two stages (GPT-2's tied ``wte``/``lm_head``) get
  their gradients summed between the owning stages before the optimizer
  step, and are broadcast once at build time.
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

    ``to_empty`` creates new Parameter objects; an ``optimizer`` built over the meta
    parameters is re-pointed at them (matched by parameter name)."""
    if not any(t.is_meta for t in list(module.parameters()) + list(module.buffers())):
        return False
    old = {id(p): n for n, p in module.named_parameters(remove_duplicate=False)}
    module.to_empty(device=device)
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


class P2P:
    """Point-to-point transport between adjacent stages (global ranks)."""

    def __init__(self, prev: Optional[int], nxt: Optional[int], group, device):
        self.prev, self.next, self.group, self.device = prev, nxt, group, device
        self.pending = []
        # RCCL moves device tensors directly over xGMI; a gloo group (CPU tier, or several
        # ranks sharing one GPU in tests) stages device tensors through host memory.
        backend = dist.get_backend(group) if dist.is_initialized() else "gloo"
        self.host_staged = backend == "gloo" and torch.device(device).type == "cuda"
        self.buf_device = torch.device("cpu") if self.host_staged else torch.device(device)

    def _run(self, ops):
        if not ops:
            return
        reqs = dist.batch_isend_irecv(ops)
        for r in reqs:
            r.wait()

    def exchange(self, send_t=None, send_to=None, recv_shape=None, recv_dtype=None, recv_from=None):
        ops = []
        out = None
        if send_t is not None and send_to is not None:
            send_t = send_t.contiguous()
            if self.host_staged:
                send_t = send_t.cpu()
            ops.append(dist.P2POp(dist.isend, send_t, send_to, self.group))
            self.pending.append(send_t)
        if recv_shape is not None and recv_from is not None:
            out = torch.empty(recv_shape, dtype=recv_dtype, device=self.buf_device)
            ops.append(dist.P2POp(dist.irecv, out, recv_from, self.group))
        self._run(ops)
        if out is not None and self.host_staged:
            out = out.to(self.device)
        return out

    def send_meta(self, t: torch.Tensor, to: int):
        hdr = torch.zeros(10, dtype=torch.int64, device=self.buf_device)
        hdr[0] = t.dim()
        hdr[1] = _DT_CODE[t.dtype]
        hdr[2:2 + t.dim()] = torch.tensor(t.shape, dtype=torch.int64)
        self._run([dist.P2POp(dist.isend, hdr, to, self.group)])

    def recv_meta(self, frm: int):
        hdr = torch.empty(10, dtype=torch.int64, device=self.buf_device)
        self._run([dist.P2POp(dist.irecv, hdr, frm, self.group)])
        h = hdr.tolist()
        return tuple(int(v) for v in h[2:2 + h[0]]), _CODE_DT[h[1]]

    def flush(self):
        self.pending.clear()


class PipelineEngine:
    """Runs one pipeline stage of a (dp x pp) mesh; ``train_step`` = fwd + bwd of all microbatches."""

    def __init__(self, stage_module: StageModule, *, stage: int, nstages: int, groups: rt.ProcessGroups,
                 microbatches: int, schedule: str, loss_fn: Callable, dp_engine: DataParallel,
                 cast_dtype, tied: List[tuple], param_names: Dict[int, str], buffer_refs=()):
        self.module = stage_module
        self.stage, self.nstages = stage, nstages
        self.groups = groups
        self.M = microbatches
        self.schedule = schedule
        self.loss_fn = loss_fn
        self.dp = dp_engine
        self.sync = "grads"
        self.cast_dtype = cast_dtype
        self.tied = tied                      # [(param, group)] on this rank
        self.param_names = param_names
        self.buffer_refs = list(buffer_refs)   # (original name, owner module, local name)
        dev = rt.device()
        prev = groups.pp_ranks[stage - 1] if stage > 0 else None
        nxt = groups.pp_ranks[stage + 1] if stage < nstages - 1 else None
        self.p2p = P2P(prev, nxt, groups.pp_group, dev)
        self.program = native_runtime.pipeline_program(schedule, stage, nstages, microbatches)
        # A collective over every group first: RCCL communicators exist before the first
        # batched send/recv, which must not be a group's first operation.
        if dist.is_initialized():
            probe = torch.zeros(1, device=dev)
            for g in (groups.pp_group, groups.dp_group):
                comm.all_reduce(probe, "sum", group=g)
            for _, g in tied:
                comm.all_reduce(probe, "sum", group=g)
        self._sig = None
        self._in_meta = None     # (shape, dtype) of the activation this stage receives
        self._out_meta = None    # (shape, dtype) of the activation this stage sends
        self.last_loss = None

    @property
    def is_first(self):
        return self.stage == 0

    @property
    def is_last(self):
        return self.stage == self.nstages - 1

    # ------------------------------------------------------------ training
    def train_step(self, inputs: torch.Tensor, targets: Optional[torch.Tensor] = None):
        """Forward + backward of every microbatch of this stage; returns the mean loss on the last stage."""
        self.module.train()
        M = self.M
        xs = list(inputs.chunk(M)) if self.is_first else [None] * M
        ts = list(targets.chunk(M)) if (self.is_last and targets is not None) else [None] * M
        if len(xs) != M or len(ts) != M:
            raise ValueError(f"batch of {inputs.shape[0]} does not split into {M} microbatches")
        sig = (tuple(inputs.shape), inputs.dtype)
        new_sig = sig != self._sig
        self._sig = sig
        acts_in: Dict[int, torch.Tensor] = {}
        acts_out: Dict[int, torch.Tensor] = {}
        losses: Dict[int, torch.Tensor] = {}
        grads_in: Dict[int, torch.Tensor] = {}
        total = torch.zeros((), device=rt.device(), dtype=torch.float32) if self.is_last else None
        pr, nx = self.p2p.prev, self.p2p.next

        def recv_fwd(m):
            if self.is_first:
                x = _cast_inputs(xs[m], self.cast_dtype, False)
            else:
                if m == 0 and new_sig:
                    self._in_meta = self.p2p.recv_meta(pr)
                shape, dt = self._in_meta
                x = self.p2p.exchange(recv_shape=shape, recv_dtype=dt, recv_from=pr)
                x.requires_grad_(x.is_floating_point())
            acts_in[m] = x

        def fwd(m):
            y = self.module(acts_in[m])
            if self.is_last:
                loss = self.loss_fn(y, ts[m]) / M
                losses[m] = loss
                total.add_(loss.detach().float())
            else:
                acts_out[m] = y
                if m == 0 and new_sig:
                    self._out_meta = (tuple(y.shape), y.dtype)

        def send_fwd(m):
            if self.is_last:
                return
            y = acts_out[m]
            if m == 0 and new_sig:
                self.p2p.send_meta(y, nx)
            self.p2p.exchange(send_t=y.detach(), send_to=nx)

        def recv_bwd(m):
            if self.is_last:
                return
            shape, dt = self._out_meta
            grads_in[m] = self.p2p.exchange(recv_shape=shape, recv_dtype=dt, recv_from=nx)

        def bwd(m):
            last_mb = m == M - 1
            ctx = self.dp.no_sync() if not last_mb else _null()
            with ctx:
                if self.is_last:
                    losses.pop(m).backward()
                else:
                    torch.autograd.backward(acts_out.pop(m), grad_tensors=grads_in.pop(m))

        def send_bwd(m):
            x = acts_in.pop(m)
            if self.is_first:
                return
            g = x.grad if x.grad is not None else torch.zeros_like(x)
            self.p2p.exchange(send_t=g, send_to=pr)

        for op, a, b in self.program:
            if op == "RECV_FWD":
                recv_fwd(a)
            elif op == "FWD":
                fwd(a)
            elif op == "SEND_FWD":
                send_fwd(a)
            elif op == "RECV_BWD":
                recv_bwd(a)
            elif op == "BWD":
                bwd(a)
            elif op == "SEND_BWD":
                send_bwd(a)
            elif op == "SEND_FWD_RECV_BWD":
                if self.is_last:
                    continue
                y = acts_out[a]
                shape, dt = self._out_meta
                grads_in[b] = self.p2p.exchange(send_t=y.detach(), send_to=nx, recv_shape=shape, recv_dtype=dt,
                                                recv_from=nx)
            elif op == "SEND_BWD_RECV_FWD":
                x = acts_in.pop(a)
                if self.is_first:
                    recv_fwd(b)
                    continue
                g = x.grad if x.grad is not None else torch.zeros_like(x)
                shape, dt = self._in_meta
                nxt_x = self.p2p.exchange(send_t=g, send_to=pr, recv_shape=shape, recv_dtype=dt, recv_from=pr)
                nxt_x.requires_grad_(nxt_x.is_floating_point())
                acts_in[b] = nxt_x
        self.p2p.flush()
        self.last_loss = total
        return total

    # -------------------------------------------------- optimizer protocol
    def finalize_grads(self):
        self.dp.finalize_grads()
        for p, group in self.tied:
            bk, off, _ = self.dp.space.param_info[id(p)]
            buf = self.dp.space.grad_buffer(bk)
            comm.all_reduce(buf[off:off + p.numel()], "sum", group=group)

    def after_step(self):
        self.dp.after_step()

    def comm_metrics(self) -> dict:
        """DP all-reduce numbers of this stage plus the schedule's analytic bubble fraction
        ((S-1)/(M+S-1) for GPipe and 1F1B with S stages and M microbatches)."""
        out = self.dp.comm_metrics()
        out["bubble_fraction"] = (self.nstages - 1) / (self.M + self.nstages - 1)
        return out

    # ------------------------------------------------------------ inference
    @torch.no_grad()
    def forward_step(self, inputs: torch.Tensor) -> Optional[torch.Tensor]:
        """Pipelined forward only (GPipe order); returns the full output on the last stage."""
        self.module.eval()
        M = self.M
        xs = list(inputs.chunk(M)) if self.is_first else [None] * M
        outs = []
        pr, nx = self.p2p.prev, self.p2p.next
        for m in range(M):
            if self.is_first:
                x = _cast_inputs(xs[m], self.cast_dtype, False)
            else:
                shape, dt = self.p2p.recv_meta(pr)
                x = self.p2p.exchange(recv_shape=shape, recv_dtype=dt, recv_from=pr)
            y = self.module(x)
            if self.is_last:
                outs.append(y)
            else:
                self.p2p.send_meta(y, nx)
                self.p2p.exchange(send_t=y, send_to=nx)
        self.p2p.flush()
        return torch.cat(outs) if outs else None

    def state_dict(self):
        """This stage's parameters under their ORIGINAL model names."""
        out = {}
        for p in self.module.parameters():
            name = self.param_names.get(id(p))
            if name is not None:
                out[name] = p
        return out

    def named_buffers(self):
        for name, owner, local in self.buffer_refs:
            yield name, owner.get_buffer(local)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def build_pipeline(model: nn.Module, optimizer, cfg: Config, plan, loss_fn: Optional[Callable] = None):
    """Cut ``model`` along ``plan`` and return ``(PipelineEngine, stage_optimizer)`` for this rank."""
    from ..api import _is_fused, build_space, prepare_model

    rt.init(timeout_s=cfg.timeout_s)
    world = rt.get_world_size()
    mesh = rt.Mesh(dp=plan.dp, pp=plan.pp, tp=1)
    if mesh.size != world:
        raise ValueError(f"plan {plan.dp}x{plan.pp} does not match world size {world}")
    groups = rt.ProcessGroups(mesh)
    stage = groups.pp_idx
    lo, hi = plan.bounds[stage], plan.bounds[stage + 1]
    layers = plan.spine.layers[lo:hi]
    pmap, bmap = original_names(model, layers)
    stage_mod = StageModule(layers, plan.checkpoint[lo:hi])
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

    # tied parameters: which stages hold each shared parameter
    owners: Dict[int, List[int]] = {}
    objs = {}
    for s in range(plan.pp):
        for layer in plan.spine.layers[plan.bounds[s]:plan.bounds[s + 1]]:
            for p in layer.parameters():
                lst = owners.setdefault(id(p), [])
                if s not in lst:
                    lst.append(s)
                objs[id(p)] = p
    tied_sets = [(pid, sts) for pid, sts in owners.items() if len(sts) > 1]
    tied_local = []
    for pid, sts in tied_sets:  # every rank creates every group, same order
        for d in range(plan.dp):
            ranks = [mesh.rank_of(d, s, 0) for s in sts]
            grp = dist.new_group(ranks) if dist.is_initialized() else None
            if rt.get_rank() in ranks:
                tied_local.append((objs[pid], grp, ranks[0]))

    dtype, dtype_of, cl = prepare_model(stage_mod, cfg, dev)
    names, buffer_refs = stage_names(layers, pmap, bmap)
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
                             broadcast_buffers=cfg.broadcast_buffers, find_unused=True, sync_comm=cfg.sync_comm)
    engine = PipelineEngine(stage_mod, stage=stage, nstages=plan.pp, groups=groups, microbatches=plan.microbatches,
                            schedule=cfg.schedule, loss_fn=loss_fn, dp_engine=dp_engine, cast_dtype=dtype,
                            tied=[(p, g) for p, g, _ in tied_local], param_names=names,
                            buffer_refs=buffer_refs)
    engine.plan = plan
    if optimizer is not None:
        if not _is_fused(optimizer):
            raise TypeError("pipeline engine needs a madnn fused optimizer (FusedSGD / FusedAdam)")
        optimizer.bind(space)
        optimizer.grad_source = engine
    get_logger().info("madnn pp: stage %d/%d layers [%d, %d) dp=%d microbatches=%d schedule=%s tied=%d",
                      stage, plan.pp, lo, hi, plan.dp, plan.microbatches, cfg.schedule, len(tied_local))
    return engine, optimizer
