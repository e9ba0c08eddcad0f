"""Per-layer cost model: FLOPs, bytes moved, parameters, activation memory,
and (optionally) measured forward/backward time with HIP events.

Reference: the only cost signal in TorchAD-NN is a dead probe that times
10 x (forward, backward, synchronizeGradients) (datamodule.lua:280-303,
call commented out at :42) plus a size-only heuristic (datamodule.lua:68-78).
Here every layer of the traced spine is costed analytically on the META
device — no weights are materialised, so an 8B-parameter model is costed on a
laptop — by running it under a dispatch mode that counts matmul/conv/attention
FLOPs (``torch.utils.flop_counter``) and the bytes every op writes.  On a GPU,
``measure()`` replaces the analytic times with HIP-event timings.
"""
from __future__ import annotations

import os

import math
from dataclasses import dataclass, field
from typing import Any, List, Optional

import torch
from torch import nn
from torch.func import functional_call
from torch.utils._python_dispatch import TorchDispatchMode
from torch.utils.flop_counter import FlopCounterMode

from .hw import Machine, load
from .trace import Spine


@dataclass
class LayerCost:
    name: str
    params: int                 # parameters owned by this layer (shared ones counted where first seen)
    shared_params: int          # parameters also used by another layer (tied weights)
    flops: float                # forward FLOPs per sample
    act_bytes: float            # bytes written by forward ops per sample (~ saved-activation memory)
    out_bytes: float            # boundary tensor bytes per sample (what a stage sends)
    out_shape: tuple = ()
    out_dtype: Any = None
    fwd_s: float = 0.0          # per-sample forward time estimate (or measurement)
    bwd_s: float = 0.0
    measured: bool = False
    fixed_s: float = 0.0        # per-CALL fwd+bwd cost independent of the batch (launches, small-batch
    #                             under-occupancy): one microbatch of n samples takes fixed_s + n * time_s
    nops: int = 0               # ops dispatched by one forward (launch-count proxy)

    @property
    def time_s(self) -> float:
        return self.fwd_s + self.bwd_s

    def call_s(self, n: float) -> float:
        """fwd+bwd seconds of one call on ``n`` samples."""
        return self.fixed_s + n * self.time_s


class _BytesMode(TorchDispatchMode):
    """Counts bytes of every op output (excluding views)."""

    def __init__(self):
        super().__init__()
        self.bytes = 0
        self.ops = 0

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = getattr(func, "__name__", "")
        if not any(v in name for v in ("view", "alias", "expand", "as_strided", "permute", "transpose", "detach",
                                       "t.default", "unsqueeze", "squeeze", "slice", "select", "split")):
            self.ops += 1
            for t in (out if isinstance(out, (list, tuple)) else (out,)):
                if isinstance(t, torch.Tensor):
                    self.bytes += t.numel() * t.element_size()
        return out


def _meta_state(layer: nn.Module, dtype: Optional[torch.dtype]):
    st = {}
    for n, p in layer.named_parameters(remove_duplicate=False):
        dt = dtype if (dtype is not None and p.is_floating_point()) else p.dtype
        st[n] = torch.empty(p.shape, dtype=dt, device="meta")
    for n, b in layer.named_buffers(remove_duplicate=False):
        st[n] = torch.empty(b.shape, dtype=b.dtype, device="meta")
    return st


def _to_meta(x, dtype):
    if isinstance(x, torch.Tensor):
        dt = dtype if (dtype is not None and x.is_floating_point()) else x.dtype
        return torch.empty(x.shape, dtype=dt, device="meta")
    return x


class _FlashSDPA:
    """Cost stand-in for F.scaled_dot_product_attention during meta estimation.

    On MI355X attention runs as a fused flash kernel (no S x S matrix in HBM), but
    on the meta device SDPA would decompose into the math path and count the
    score matrix; this replaces it with the flash cost: 4*B*H*Sq*Sk*D FLOPs
    (halved when causal) and only the output tensor written."""

    def __init__(self):
        self.flops = 0.0
        self._orig = None

    def __call__(self, q, k, v, attn_mask=None, dropout_p=0.0, is_causal=False, scale=None, enable_gqa=False):
        b, h, sq, d = q.shape
        sk = k.shape[-2]
        f = 4.0 * b * h * sq * sk * d
        self.flops += f / 2 if is_causal else f
        return torch.empty(b, h, sq, v.shape[-1], dtype=q.dtype, device=q.device)

    def __enter__(self):
        import torch.nn.functional as F

        self._orig = F.scaled_dot_product_attention
        F.scaled_dot_product_attention = self
        return self

    def __exit__(self, *exc):
        import torch.nn.functional as F

        F.scaled_dot_product_attention = self._orig
        return False


def estimate(spine: Spine, example_input: torch.Tensor, dtype: Optional[torch.dtype] = torch.bfloat16,
             machine: Optional[Machine] = None) -> List[LayerCost]:
    """Analytic per-sample costs of every spine layer (meta device, no allocation)."""
    hw = machine or load()
    if example_input.dim() > 0 and example_input.shape[0] == 1:
        # costs are per sample; two samples keep training-mode BatchNorm (one value per channel
        # after a global pool) valid
        example_input = example_input.expand(2, *example_input.shape[1:])
    batch = example_input.shape[0] if example_input.dim() > 0 else 1
    x = _to_meta(example_input, dtype)
    seen = {}
    for i, layer in enumerate(spine.layers):
        for p in layer.parameters():
            seen.setdefault(id(p), []).append(i)
    costs = []
    counted = set()
    for i, (layer, name) in enumerate(zip(spine.layers, spine.names)):
        own = shared = 0
        for p in layer.parameters():
            if len(seen[id(p)]) > 1:
                shared += p.numel()
            if id(p) not in counted:
                own += p.numel()
                counted.add(id(p))
        st = _meta_state(layer, dtype)
        fc = FlopCounterMode(display=False)
        bm = _BytesMode()
        with torch.no_grad(), _FlashSDPA() as attn, fc, bm:
            y = functional_call(layer, st, (x,))
        flops = (fc.get_total_flops() + attn.flops) / batch
        act = bm.bytes / batch
        out_b = y.numel() * y.element_size() / batch
        eff_flops = hw.bf16_tflops * 1e12 if (dtype in (torch.bfloat16, torch.float16)) else hw.fp32_tflops * 1e12
        fwd = flops / eff_flops + 2.0 * act / (hw.hbm_tbps * 1e12)  # write + one re-read of every output
        # forward launches + ~2x as many in backward
        fixed = 3.0 * bm.ops * hw.kernel_launch_us * 1e-6
        costs.append(LayerCost(name=name, params=own, shared_params=shared, flops=flops, act_bytes=act,
                               out_bytes=out_b, out_shape=tuple(y.shape[1:]), out_dtype=y.dtype,
                               fwd_s=fwd, bwd_s=2.0 * fwd, fixed_s=fixed, nops=bm.ops))
        x = y
    return costs


def measure(spine: Spine, example_input: torch.Tensor, costs: List[LayerCost], iters: int = 3) -> List[LayerCost]:
    """Replace analytic times with HIP-event timings of each layer (fwd and fwd+bwd).

    Requires the spine's parameters to live on the GPU; the example input's batch
    is used as is (per-sample numbers are divided by it)."""
    if not torch.cuda.is_available():
        return costs
    batch = example_input.shape[0]
    x = example_input
    for layer, c in zip(spine.layers, costs):
        xin = x.detach().requires_grad_(x.is_floating_point())
        for _ in range(2):
            y = layer(xin)
        start, mid, end = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        fw = bw = 0.0
        for _ in range(iters):
            start.record()
            y = layer(xin)
            mid.record()
            if y.requires_grad:
                y.backward(torch.ones_like(y))
            end.record()
            end.synchronize()
            fw += start.elapsed_time(mid)
            bw += mid.elapsed_time(end)
        c.fwd_s = fw / iters / 1e3 / batch
        c.bwd_s = bw / iters / 1e3 / batch
        c.measured = True
        x = y.detach()
        for p in layer.parameters():
            p.grad = None
    return costs


def layer_signature(layer: nn.Module) -> tuple:
    """Layers with equal signatures (type + parameter shapes/dtypes) cost the same: the
    repeated blocks of a transformer are measured once."""
    return (type(layer).__name__,
            tuple((n, tuple(p.shape), str(p.dtype)) for n, p in layer.named_parameters(remove_duplicate=False)))


def _replica(layer: nn.Module, device, dtype):
    """A private, initialised copy of ``layer`` on ``device`` in madnn's compute layout
    (compute-dtype weights, fp32 norm parameters, channels_last convolutions)."""
    import copy

    from ..api import _has_conv, _norm_param_ids

    rep = copy.deepcopy(layer)
    if any(t.is_meta for t in list(rep.parameters()) + list(rep.buffers())):
        from ..parallel.pp import materialize_

        materialize_(rep, device)
    rep.to(device)
    keep = _norm_param_ids(rep)
    with torch.no_grad():
        for p in rep.parameters():
            if p.is_floating_point() and id(p) not in keep and dtype is not None:
                p.data = p.data.to(dtype)
    cl = device.type == "cuda" and _has_conv(rep)
    if cl:
        rep.to(memory_format=torch.channels_last)
    rep.train()
    return rep, cl


def _layer_input(i, layer_costs, example_input, b, dtype, dev):
    if i == 0:
        idx = torch.arange(b) % max(example_input.shape[0], 1)
        x = example_input[idx].to(dev)
        if x.is_floating_point():
            x = x.to(dtype or x.dtype)
        return x
    prev = layer_costs[i - 1]
    odt = prev.out_dtype or dtype
    if odt is not None and not odt.is_floating_point:
        return torch.zeros((b,) + tuple(prev.out_shape), dtype=odt, device=dev)
    return torch.randn((b,) + tuple(prev.out_shape), dtype=odt, device=dev)


def _time_call(fn, xin, iters: int):
    """(fwd ms, bwd ms) of ``fn(xin)`` averaged over ``iters`` after two warm-up calls."""
    for _ in range(2):
        y = fn(xin)
        if y.requires_grad:
            y.backward(torch.ones_like(y))
    if xin.device.type != "cuda":      # host tensors (CPU jobs): wall clock
        import time

        fw = bw = 0.0
        for _ in range(iters):
            t0 = time.perf_counter()
            y = fn(xin)
            t1 = time.perf_counter()
            if y.requires_grad:
                y.backward(torch.ones_like(y))
            fw += (t1 - t0) * 1e3
            bw += (time.perf_counter() - t1) * 1e3
        return fw / iters, bw / iters
    start, mid, end = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    fw = bw = 0.0
    for _ in range(iters):
        start.record()
        y = fn(xin)
        mid.record()
        if y.requires_grad:
            y.backward(torch.ones_like(y))
        end.record()
        end.synchronize()
        fw += start.elapsed_time(mid)
        bw += mid.elapsed_time(end)
    return fw / iters, bw / iters


class MeasurementFailed(RuntimeError):
    """A layer / chain timing failed on this rank or on a peer; every rank of the group raises it
    together (the planner then uses analytic costs everywhere)."""


def measure_layers(spine: Spine, example_input: torch.Tensor, costs: List[LayerCost], *, batch: Optional[int] = None,
                   dtype: Optional[torch.dtype] = torch.bfloat16, iters: int = 3,
                   device: Optional[torch.device] = None, group=None, two_point: bool = True) -> List[LayerCost]:
    """Replace the analytic times of ``costs`` with HIP-event timings on this GPU.

    Every DISTINCT layer (:func:`layer_signature` + input shape) is copied once onto the
    device -- a meta-device layer is materialised -- and its forward and forward+backward are
    timed at ``batch`` samples and (``two_point``) at a quarter of it, giving a per-call fixed
    cost and a per-sample slope (``LayerCost.fixed_s`` / ``time_s``): the planner needs both to
    price small pipeline microbatches, whose GEMMs run far below the large-batch rate.  A
    24-block transformer costs three measurements and an 8B model never needs to exist whole.

    With a process group (``group``) of W > 1 ranks the distinct layers are dealt round-robin:
    every rank times its share on its own GPU concurrently and the results are all-gathered,
    so no rank idles while one GPU times the whole model.  Returns ``costs`` unchanged without
    a GPU.  This is the working version of the reference's dead ``comm_speed`` probe
    (datamodule.lua:280-303)."""
    if device is None and not torch.cuda.is_available():
        return costs
    import torch.distributed as dist

    from .. import runtime as rt

    multi = dist.is_available() and dist.is_initialized() and rt.get_world_size(group) > 1
    me, world = (rt.get_rank(group), rt.get_world_size(group)) if multi else (0, 1)
    mine = {}
    err = None
    keys, first, distinct = [], {}, []
    try:
        # setup, timing and (below) the fit all end in MeasurementFailed on every rank, never in
        # an exception some ranks raise while their peers wait in a collective
        dev = device or torch.device("cuda", torch.cuda.current_device())
        b = int(batch or max(example_input.shape[0], 1))
        b2 = max(b // 4, 1) if two_point and b >= 4 else None
        for i, layer in enumerate(spine.layers):
            if i == 0:
                in_key = ("input", tuple(example_input.shape[1:]), str(example_input.dtype))
            else:
                in_key = (tuple(costs[i - 1].out_shape), str(costs[i - 1].out_dtype))
            key = (layer_signature(layer), in_key)
            keys.append(key)
            first.setdefault(key, i)
        distinct = sorted(first, key=lambda k: first[k])
        for j, key in enumerate(distinct):
            if j % world != me:
                continue
            i = first[key]
            rep, cl = _replica(spine.layers[i], dev, dtype)
            res = []
            for n in ([b] + ([b2] if b2 else [])):
                x = _layer_input(i, costs, example_input, n, dtype, dev)
                if cl and x.dim() == 4:
                    x = x.contiguous(memory_format=torch.channels_last)
                # the model input needs no gradient (a conv stem's data grad is a large, slow pass
                # the training step never runs); every later layer's input does
                xin = x.detach().requires_grad_(x.is_floating_point() and i > 0)
                res.append((n,) + _time_call(rep, xin, iters))
                del x, xin
            for p in rep.parameters():
                p.grad = None
            del rep
            mine[j] = res
        if os.environ.get("MADNN_FAULT_MEASURE") == str(me):   # test hook: this rank's timing fails
            raise RuntimeError(f"injected layer-measurement failure on rank {me}")
    except Exception as e:  # noqa: BLE001 - decided together below
        err = e
    if multi:
        from .. import comm

        # every rank learns whether ALL measured before anyone enters the gather: a rank that
        # failed alone would otherwise leave its peers blocked in all_gather_object
        if not comm.all_agree(err is None, group):
            raise MeasurementFailed(f"layer measurement failed on some rank ({err or 'a peer'})")
    elif err is not None:
        raise MeasurementFailed(str(err)) from err
    if multi:
        gathered = [None] * world
        dist.all_gather_object(gathered, mine, group=group)
        for g in gathered:
            mine.update(g)
    try:
        fitted = _fit_measurements(distinct, mine)
    except Exception as e:  # noqa: BLE001 - every rank fits the same gathered numbers: same outcome
        raise MeasurementFailed(f"fitting the layer timings failed ({e})") from e
    for key, c in zip(keys, costs):
        c.fwd_s, c.bwd_s, c.fixed_s = fitted[key]
        c.measured = True
    torch.cuda.empty_cache()
    return costs


def _fit_measurements(distinct, mine) -> dict:
    """Per distinct layer: (fwd s/sample, bwd s/sample, fixed s/call) from its one or two timings."""
    fitted = {}
    for j, key in enumerate(distinct):
        res = mine[j]
        (n1, f1, k1) = res[0]
        fwd_ps, bwd_ps, fixed = f1 / n1, k1 / n1, 0.0
        if len(res) > 1:
            (n2, f2, k2) = res[1]
            # t(n) = fixed + n * slope through the two points; a component whose time did not grow
            # with the batch (launch-bound noise at the small size, or a small part of the layer,
            # e.g. a loss node whose gradient the forward already formed) keeps the large batch's
            # per-sample rate instead of a zero slope: no layer is free per sample
            slope_f = (f1 - f2) / (n1 - n2) if n1 != n2 else 0.0
            slope_b = (k1 - k2) / (n1 - n2) if n1 != n2 else 0.0
            slope_f = slope_f if slope_f > 0 else f1 / n1
            slope_b = slope_b if slope_b > 0 else k1 / n1
            if slope_f + slope_b > 0:
                fixed = max((f1 + k1) - n1 * (slope_f + slope_b), 0.0)
                fwd_ps, bwd_ps = slope_f, slope_b
        fitted[key] = (fwd_ps / 1e3, bwd_ps / 1e3, fixed / 1e3)
    return fitted


def measure_chain(spine: Spine, example_input: torch.Tensor, costs: List[LayerCost], *, batch: int,
                  dtype: Optional[torch.dtype] = torch.bfloat16, iters: int = 3,
                  device: Optional[torch.device] = None, saved: Optional[dict] = None) -> Optional[float]:
    """fwd+bwd seconds of the WHOLE spine, layer after layer as the model runs them, at
    ``batch`` samples -- the one-step calibration of the per-layer sum (isolated layer timings
    miss the cache/launch interplay between neighbours).  With ``saved`` (a dict), also the
    device bytes one forward keeps alive for the backward (``saved["bytes"]``).  None without
    a GPU."""
    if not torch.cuda.is_available():
        return None
    dev = device or torch.device("cuda", torch.cuda.current_device())
    reps = [_replica(layer, dev, dtype) for layer in spine.layers]
    cl = any(c for _, c in reps)

    def chain(x):
        for rep, _ in reps:
            x = rep(x)
        return x

    x = _layer_input(0, costs, example_input, batch, dtype, dev)
    if cl and x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
    xin = x.detach()  # the model input: no data gradient, as in the training step
    fw, bw = _time_call(chain, xin, iters)
    if saved is not None and dev.type == "cuda":
        # what one forward keeps alive for its backward: the saved activations, measured
        torch.cuda.synchronize(dev)
        before = torch.cuda.memory_allocated(dev)
        y = chain(xin)
        torch.cuda.synchronize(dev)
        saved["bytes"] = float(torch.cuda.memory_allocated(dev) - before)
        if y.requires_grad:
            y.backward(torch.ones_like(y))
        del y
    del reps, x, xin
    torch.cuda.empty_cache()
    return (fw + bw) / 1e3


def param_state_bytes(params: int, optimizer: str = "adam", compute_bytes: int = 2) -> float:
    """Bytes per parameter in madnn's layout: bf16 model + bf16 grad + fp32 master
    + fp32 flat reduce buffer + optimizer state (SGD momentum 4 B, Adam 8 B)."""
    opt = 8 if optimizer == "adam" else 4
    master = 4 if compute_bytes < 4 else 0
    return params * (compute_bytes + compute_bytes + master + 4 + opt)


@dataclass
class StageEstimate:
    layers: tuple
    time_per_sample_s: float
    param_bytes: float
    act_bytes_per_sample: float
    out_bytes_per_sample: float
    params: int = 0
    notes: list = field(default_factory=list)


def stage_estimate(costs: List[LayerCost], lo: int, hi: int, optimizer: str = "adam",
                   checkpoint: bool = False) -> StageEstimate:
    seg = costs[lo:hi]
    t = sum(c.time_s for c in seg)
    params = sum(c.params + (c.shared_params if lo > 0 and c.shared_params else 0) for c in seg)
    if checkpoint:
        t += sum(c.fwd_s for c in seg)  # recompute forward in backward
        act = sum(c.out_bytes for c in seg) + max((c.act_bytes for c in seg), default=0.0)
    else:
        act = sum(c.act_bytes for c in seg)
    return StageEstimate((lo, hi), t, param_state_bytes(params, optimizer), act, seg[-1].out_bytes if seg else 0.0,
                         params)


def divisors(n: int):
    return [d for d in range(1, n + 1) if n % d == 0]


def ceil_div(a, b):
    return int(math.ceil(a / b))
