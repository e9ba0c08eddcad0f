"""Tensor (model) parallelism: column/row-parallel Linear with exact conjugate
collectives, plus the reference's ``MP*`` layer names with corrected math.

Reference (nodemodule.lua): ``MPInitialLinear`` / ``MPBaseLinear`` shard the
LAST (feature) dimension of the input across all ranks (weight ``[o, i/W]``),
all-reduce the partial outputs, and in backward all-reduce (sum) the disjoint
input-gradient shards; ``MPTanh`` narrows its saved output during the first
backward pass and tiles the local gradient shard W times; the bias is added on
every rank before the sum.  The math is exact only for W = 1 (SURVEY A-9..A-12).

Here the same layers are autograd-native with the intended semantics:

* row-parallel:  x_r = shard(x)  [bwd: all-gather of the input-grad shards]
                 y   = all_reduce(x_r W_r^T) + b   [bias added once, after the sum]
* column-parallel: x replicated [bwd: all-reduce of dx], y_r = x W_r^T + b_r,
                 optional all-gather of the output (bwd: take the own shard)
* ``MPTanh`` is a plain tanh: the row-parallel backward already returns the
  full input gradient, so no narrowing/tiling is needed (the reference's
  ``syncTanh``/``syncReshape`` flags are accepted and ignored).

All TP ranks must see identical inputs (the reference's DP and MP conflict on
this, A-15; in madnn the TP group is a sub-group of the mesh).
"""
from __future__ import annotations

import os

import math
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

from .. import comm
from .. import runtime as rt

_DEBUG = {"shapes": False}


def set_debug_shapes(on: bool = True) -> None:
    """Print per-layer input/output/grad shapes (reference ``printDims``, nodemodule.lua:3)."""
    _DEBUG["shapes"] = on


def _dbg(tag, *ts):
    if _DEBUG["shapes"]:
        print(f"[madnn tp r{rt.get_rank()}] {tag}: " + ", ".join(str(tuple(t.shape)) for t in ts if t is not None))


def _world(group) -> int:
    return rt.get_world_size(group)


def _rank(group) -> int:
    return rt.get_rank(group)


def _gather_last(x: torch.Tensor, group) -> torch.Tensor:
    """Concatenate the ranks' shards along the LAST dim.  RCCL gathers rank-major ([W, ..., k]);
    the last-dim layout interleaves the ranks inside every row, so exactly one re-layout pass
    (a strided copy of the [W, rows, k] buffer into [rows, W, k]) produces the output -- no
    per-rank views and no cat."""
    w = _world(group)
    if w == 1:
        return x
    x = x.contiguous()
    buf = torch.empty((w,) + tuple(x.shape), dtype=x.dtype, device=x.device)
    comm.all_gather_into(buf.view(w * x.shape[0], *x.shape[1:]) if x.dim() > 0 else buf, x, group=group)
    if x.dim() == 0:
        return buf
    return buf.movedim(0, -2).reshape(*x.shape[:-1], w * x.shape[-1])


def _shard_last(x: torch.Tensor, group) -> torch.Tensor:
    w = _world(group)
    if w == 1:
        return x
    n = x.shape[-1]
    if n % w:
        raise ValueError(f"last dim {n} not divisible by TP size {w}")
    k = n // w
    return x.narrow(-1, _rank(group) * k, k).contiguous()


class _Scatter(torch.autograd.Function):
    """fwd: own shard of the last dim; bwd: all-gather of the shard grads."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _shard_last(x, group)

    @staticmethod
    def backward(ctx, g):
        return _gather_last(g, ctx.group), None


class _Gather(torch.autograd.Function):
    """fwd: all-gather along the last dim; bwd: own shard."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _gather_last(x, group)

    @staticmethod
    def backward(ctx, g):
        return _shard_last(g, ctx.group), None


class _Reduce(torch.autograd.Function):
    """fwd: sum all-reduce; bwd: identity (the output is replicated)."""

    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous().clone()
        comm.all_reduce(x, "sum", group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _Copy(torch.autograd.Function):
    """fwd: identity; bwd: sum all-reduce (a replicated input feeding sharded weights)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        comm.all_reduce(g, "sum", group=ctx.group)
        return g, None


class RowParallelLinear(nn.Module):
    """y = x W^T + b with W split along its INPUT dim (``[out, in/W]`` per rank)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, input_is_parallel: bool = False,
                 group=None, device=None, dtype=None):
        super().__init__()
        w = _world(group)
        if in_features % w:
            raise ValueError(f"in_features {in_features} not divisible by TP size {w} (reference assert, "
                             "nodemodule.lua:36,88)")
        self.in_features, self.out_features = in_features, out_features
        self.group, self.input_is_parallel = group, input_is_parallel
        self.local_in = in_features // w
        self.weight = nn.Parameter(torch.empty(out_features, self.local_in, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.empty(out_features, device=device, dtype=dtype)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        # same distribution as nn.Linear over the FULL fan-in
        bound = 1.0 / math.sqrt(self.in_features)
        nn.init.uniform_(self.weight, -bound, bound)
        if self.bias is not None:
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        xs = x if self.input_is_parallel else _Scatter.apply(x, self.group)
        y = _Reduce.apply(F.linear(xs, self.weight), self.group)
        if self.bias is not None:
            y = y + self.bias
        _dbg("RowParallelLinear", x, xs, y)
        return y

    @torch.no_grad()
    def load_full(self, weight: torch.Tensor, bias: Optional[torch.Tensor] = None):
        """Take this rank's shard from a full ``[out, in]`` weight."""
        r = _rank(self.group)
        self.weight.copy_(weight[:, r * self.local_in:(r + 1) * self.local_in])
        if bias is not None and self.bias is not None:
            self.bias.copy_(bias)

    def extra_repr(self):
        return f"in={self.in_features} (local {self.local_in}), out={self.out_features}, tp={_world(self.group)}"


class ColumnParallelLinear(nn.Module):
    """y = x W^T + b with W split along its OUTPUT dim (``[out/W, in]`` per rank)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, gather_output: bool = True,
                 group=None, device=None, dtype=None):
        super().__init__()
        w = _world(group)
        if out_features % w:
            raise ValueError(f"out_features {out_features} not divisible by TP size {w}")
        self.in_features, self.out_features = in_features, out_features
        self.group, self.gather_output = group, gather_output
        self.local_out = out_features // w
        self.weight = nn.Parameter(torch.empty(self.local_out, in_features, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.empty(self.local_out, device=device, dtype=dtype)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        bound = 1.0 / math.sqrt(self.in_features)
        nn.init.uniform_(self.weight, -bound, bound)
        if self.bias is not None:
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        y = F.linear(_Copy.apply(x, self.group), self.weight, self.bias)
        out = _Gather.apply(y, self.group) if self.gather_output else y
        _dbg("ColumnParallelLinear", x, out)
        return out

    @torch.no_grad()
    def load_full(self, weight: torch.Tensor, bias: Optional[torch.Tensor] = None):
        r = _rank(self.group)
        self.weight.copy_(weight[r * self.local_out:(r + 1) * self.local_out])
        if bias is not None and self.bias is not None:
            self.bias.copy_(bias[r * self.local_out:(r + 1) * self.local_out])

    def extra_repr(self):
        return f"in={self.in_features}, out={self.out_features} (local {self.local_out}), tp={_world(self.group)}"


# --------------------------------------------------------------------------
# Reference-compatible layer names (nodemodule.lua), corrected semantics
# --------------------------------------------------------------------------
class MPInitialLinear(RowParallelLinear):
    """``nn.MPInitialLinear(i, o)`` (nodemodule.lua:34-73): first FC layer, full input sharded on its last dim."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, group=None):
        super().__init__(in_features, out_features, bias=bias, input_is_parallel=False, group=group)


class MPBaseLinear(RowParallelLinear):
    """``nn.MPBaseLinear(i, o)`` (nodemodule.lua:86-119): later FC layers (same math as MPInitialLinear)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, group=None):
        super().__init__(in_features, out_features, bias=bias, input_is_parallel=False, group=group)


class MPTanh(nn.Module):
    """``nn.MPTanh()`` (nodemodule.lua:132-174).  ``sync`` mirrors ``syncTanh`` and is a no-op: the
    corrected row-parallel backward already delivers the full gradient."""

    def __init__(self, sync: bool = True):
        super().__init__()
        self.sync = sync

    def forward(self, x):
        y = torch.tanh(x)
        _dbg("MPTanh", x, y)
        return y


class _Reshape(nn.Module):
    def __init__(self, *shape):
        super().__init__()
        self.shape = tuple(shape[0]) if len(shape) == 1 and isinstance(shape[0], (tuple, list)) else tuple(shape)

    def forward(self, x):
        n = 1
        for s in self.shape:
            n *= s
        batch = x.numel() // n
        y = x.reshape(batch, *self.shape) if batch > 1 or x.dim() > len(self.shape) else x.reshape(self.shape)
        _dbg(type(self).__name__, x, y)
        return y


class MPInitialReshape(_Reshape):
    """``nn.MPInitialReshape(...)`` (nodemodule.lua:186-226): reshape before the first MP linear."""


class MPBaseReshape(_Reshape):
    """``nn.MPBaseReshape(...)`` (nodemodule.lua:238-285): reshape between MP layers (``syncReshape`` no-op)."""


# --------------------------------------------------------------------------
# strategy="tp": shard the large Linear layers of an arbitrary model
# --------------------------------------------------------------------------
_ELEMENTWISE = (nn.ReLU, nn.GELU, nn.Tanh, nn.SiLU, nn.Sigmoid, nn.Dropout, nn.Identity, nn.LeakyReLU, nn.ELU)


def _eligible(m: nn.Module, w: int, min_params: int, dim: str) -> bool:
    if type(m) is not nn.Linear or m.weight.numel() < min_params:
        return False
    return (m.in_features if dim == "in" else m.out_features) % w == 0


def _column(child: nn.Linear, group, gather_output: bool) -> "ColumnParallelLinear":
    new = ColumnParallelLinear(child.in_features, child.out_features, bias=child.bias is not None,
                               gather_output=gather_output, group=group, device=child.weight.device,
                               dtype=child.weight.dtype)
    new.load_full(child.weight.detach(), child.bias.detach() if child.bias is not None else None)
    return new


def _row(child: nn.Linear, group, input_is_parallel: bool) -> "RowParallelLinear":
    new = RowParallelLinear(child.in_features, child.out_features, bias=child.bias is not None,
                            input_is_parallel=input_is_parallel, group=group, device=child.weight.device,
                            dtype=child.weight.dtype)
    new.load_full(child.weight.detach(), child.bias.detach() if child.bias is not None else None)
    return new


def _pairs_of(module: nn.Module):
    """Column -> row pairs of a module: declared by ``tensor_parallel_pairs()`` (madnn's MLPs:
    ``[(("c_fc",), "c_proj")]``, gated MLPs ``[(("gate_proj", "up_proj"), "down_proj")]``), or
    found in an ``nn.Sequential`` as Linear, elementwise activations, Linear."""
    if hasattr(module, "tensor_parallel_pairs"):
        return [(tuple(cols), row) for cols, row in module.tensor_parallel_pairs()]
    pairs = []
    if isinstance(module, nn.Sequential):
        names = [n for n, _ in module.named_children()]
        mods = [m for _, m in module.named_children()]
        i = 0
        while i < len(mods):
            if type(mods[i]) is nn.Linear:
                j = i + 1
                while j < len(mods) and isinstance(mods[j], _ELEMENTWISE):
                    j += 1
                if j < len(mods) and type(mods[j]) is nn.Linear and j > i:
                    pairs.append(((names[i],), names[j]))
                    i = j + 1
                    continue
            i += 1
    return pairs


def shard_linears(model: nn.Module, group=None, min_params: int = 1 << 20, _tied=None) -> int:
    """Shard the large Linears of ``model`` over ``group`` (returns how many were replaced).

    Column -> row PAIRS (:func:`_pairs_of`) become the Megatron pattern: the column-parallel
    layer keeps its output sharded (no gather), the elementwise activation runs on the shard,
    the row-parallel layer consumes the shard directly -- ONE all-reduce per pair forward
    (and one in backward, for the replicated input), no activation gather/scatter.  Every
    other eligible Linear becomes row-parallel on its own (scatter its input, all-reduce its
    output).  Weights are taken from the original layers.  A Linear whose weight is TIED to
    another module (GPT-2's lm_head = wte) stays replicated, keeping the tie."""
    w = _world(group)
    if _tied is None:
        cnt = {}
        for _, p in model.named_parameters(remove_duplicate=False):
            cnt[id(p)] = cnt.get(id(p), 0) + 1
        _tied = {k for k, v in cnt.items() if v > 1}
    n = 0
    paired = set()
    for cols, row in _pairs_of(model):
        cm = [getattr(model, c, None) for c in cols]
        rm = getattr(model, row, None)
        if rm is None or any(c is None for c in cm):
            continue
        if any(id(x.weight) in _tied for x in cm + [rm] if hasattr(x, "weight")):
            continue
        if all(_eligible(c, w, 0, "out") for c in cm) and _eligible(rm, w, 0, "in") and \
                sum(c.weight.numel() for c in cm) + rm.weight.numel() >= min_params:
            for name, c in zip(cols, cm):
                setattr(model, name, _column(c, group, gather_output=False))
                paired.add(name)
            setattr(model, row, _row(rm, group, input_is_parallel=True))
            paired.add(row)
            n += len(cols) + 1
    for name, child in list(model.named_children()):
        if name in paired:
            continue
        if _eligible(child, w, min_params, "in") and id(child.weight) not in _tied:
            setattr(model, name, _row(child, group, input_is_parallel=False))
            n += 1
        else:
            n += shard_linears(child, group, min_params, _tied)
    return n


def tp_norm_spec(model: nn.Module, group):
    """(groups, params to skip) for global-norm clipping under TP: shards are disjoint across
    the TP group (sum everything), replicated parameters count on TP rank 0 only."""
    if _world(group) == 1:
        return [], []
    sharded = set()
    for m in model.modules():
        if isinstance(m, ColumnParallelLinear):
            sharded.update(id(p) for p in m.parameters(recurse=False))
        elif isinstance(m, RowParallelLinear):
            sharded.add(id(m.weight))
    skip = [] if _rank(group) == 0 else [p for p in model.parameters() if p.requires_grad and id(p) not in sharded]
    return [group], skip


def apply_tensor_parallel(model: nn.Module, optimizer, cfg):
    """``distribute(model, opt, strategy="tp", tp_size=T)``.

    The world is laid out as ``dp x tp`` (``tp_size`` defaults to the world size).  Large
    Linears are sharded over each TP group; replicated parameters stay identical inside a
    TP group because its ranks see the same inputs.  With dp > 1, every parameter (shard or
    replica) is then averaged over its DP group by the bucketed DataParallel reducer — the
    DP group of a rank is the set of ranks holding the same TP shard index."""
    from ..api import _distribute_dp
    from ..utils.logging import get_logger

    rt.init(timeout_s=cfg.timeout_s)
    world = rt.get_world_size()
    tp = cfg.tp_size if cfg.tp_size and cfg.tp_size > 1 else world
    if world % tp:
        raise ValueError(f"tp_size {tp} does not divide world size {world}")
    groups = rt.ProcessGroups(rt.Mesh(dp=world // tp, pp=1, tp=tp))
    dev = rt.device()
    model.to(dev)
    with torch.no_grad():  # identical replicas before sharding: one bucketed broadcast per dtype
        from ..api import _flat_collective

        _flat_collective([p.data for p in model.parameters()], "broadcast", None, src=0)
    old = {id(p) for p in model.parameters()}
    n = shard_linears(model, groups.tp_group, int(cfg.extra.get("tp_min_params", 1 << 20)))
    if os.environ.get("MADNN_ONESHOT", "0") == "1" and dev.type == "cuda" and tp > 1:
        # K5: the row-parallel activation sums (small, latency-bound) over IPC-mapped peer buffers
        from ..comm import oneshot

        oneshot.enable_for(groups.tp_group, cap_bytes=int(cfg.extra.get("oneshot_cap", 4 << 20)))
    params = [p for p in model.parameters() if p.requires_grad]
    if optimizer is not None:
        keep = {id(q) for q in params}
        groups_o = []
        for g in optimizer.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = [p for p in g["params"] if id(p) in keep]
            if d["params"]:
                groups_o.append(d)
        new_params = [p for p in params if id(p) not in old]
        if new_params:
            if groups_o:
                groups_o[0]["params"] = groups_o[0]["params"] + new_params
            else:
                groups_o = [{"params": new_params}]
        optimizer = type(optimizer)(groups_o, **optimizer.defaults)
    get_logger().info("madnn tp: sharded %d Linear layers, mesh dp=%d x tp=%d", n, world // tp, tp)
    # ALWAYS through the flat-space engine, also without a DP axis (its group is then a
    # singleton: no collectives): bf16 compute copies with fp32 masters, the fused optimizer
    # over flat buckets and input casting apply to TP exactly as to DP
    engine, optimizer = _distribute_dp(model, optimizer, cfg, dev, group=groups.dp_group,
                                       src_rank=groups.dp_ranks[0])
    engine.groups = groups
    engine._norm_spec = tp_norm_spec(model, groups.tp_group)
    if optimizer is not None and hasattr(optimizer, "norm_spec"):
        optimizer.norm_spec = engine._norm_spec
    return engine, optimizer
