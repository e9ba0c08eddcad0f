"""Python entry points for madnn's hand-written gfx950 kernels.

Device tensors always go to the HIP kernels in ``_madnn_kernels.so``
(``torch.ops.madnn.*``); if that library is missing on a GPU box the call
raises — there is no silent eager fallback for device tensors.  CPU tensors
(the gloo test tier) use the eager reference in ``madnn.ops.reference``,
which is also the numerics oracle for the kernel tests.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path
from typing import Optional, Sequence

import torch
import torch.nn.functional as F

from . import reference

HERE = Path(__file__).resolve().parent
_KERNELS = HERE / "_madnn_kernels.so"
_lock = threading.Lock()
_loaded = {"kernels": False, "error": None}


def kernels_path() -> Path:
    return _KERNELS


class StaleKernelsError(RuntimeError):
    """The in-tree kernel library was built from different sources than the tree holds."""


def check_fresh(rebuild: bool = True) -> None:
    """Stale-binary guard: compare the build manifest's source digests with the sources.

    On a mismatch the library is rebuilt in-tree when ``rebuild`` and hipcc is present;
    otherwise (or if the rebuild leaves it stale) :class:`StaleKernelsError` names the
    changed sources -- an edited kernel never silently runs its old binary.
    ``MADNN_ALLOW_STALE=1`` skips the check (debugging a deliberately old binary)."""
    if os.environ.get("MADNN_ALLOW_STALE", "0") == "1":
        return
    from . import build as _b

    stale = _b.stale_sources()
    if not stale:
        return
    if rebuild:
        try:
            _b._hipcc()
        except RuntimeError:
            rebuild = False
    if rebuild:
        import sys

        print(f"[madnn] kernel library is stale ({', '.join(stale)}); rebuilding in-tree", file=sys.stderr)
        _b.build()
        stale = _b.stale_sources()
    if stale:
        raise StaleKernelsError(f"madnn: {_KERNELS.name} was built from other sources than the tree holds "
                                f"(changed: {', '.join(stale)}); run `python -m madnn.ops.build`")


def load_kernels(build_if_missing: bool = True) -> bool:
    """Load the HIP kernel library (building it in-tree if absent or stale and hipcc exists)."""
    with _lock:
        if _loaded["kernels"]:
            return True
        try:
            if not _KERNELS.exists() and build_if_missing:
                from .build import build

                build()
            check_fresh(rebuild=build_if_missing)
            torch.ops.load_library(str(_KERNELS))
            _loaded["kernels"] = True
            _loaded["error"] = None
        except StaleKernelsError:
            raise
        except Exception as e:  # noqa: BLE001
            _loaded["error"] = e
        return _loaded["kernels"]


def native_available() -> bool:
    return load_kernels()


def _need_native(what: str):
    if not load_kernels():
        raise RuntimeError(
            f"madnn: HIP kernel library needed for {what} on a GPU tensor could not be loaded "
            f"({_KERNELS}): {_loaded['error']!r}. Run `python -m madnn.ops.build`."
        )
    return torch.ops.madnn


def _is_dev(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


# --------------------------------------------------------------------------- K4
def bucket_pack(tensors: Sequence[torch.Tensor], flat: torch.Tensor, offsets: Sequence[int], scale: float = 1.0):
    """flat[off_i : off_i + numel_i] = tensors[i] * scale (physical order, any dense layout)."""
    if not tensors:
        return
    if _is_dev(flat):
        _need_native("bucket_pack").bucket_pack(list(tensors), flat, list(offsets), float(scale))
    else:
        reference.bucket_pack(tensors, flat, offsets, scale)


def bucket_unpack(tensors: Sequence[torch.Tensor], flat: torch.Tensor, offsets: Sequence[int], scale: float = 1.0):
    """tensors[i] = flat[off_i : off_i + numel_i] * scale (cast to each tensor's dtype)."""
    if not tensors:
        return
    if _is_dev(flat):
        _need_native("bucket_unpack").bucket_unpack(list(tensors), flat, list(offsets), float(scale))
    else:
        reference.bucket_unpack(tensors, flat, offsets, scale)


def flat_scale_cast(src: torch.Tensor, dst: torch.Tensor, scale: float = 1.0):
    if _is_dev(src):
        _need_native("flat_scale_cast").flat_scale_cast(src, dst, float(scale))
    else:
        dst.copy_(src.float().mul(scale))


# ------------------------------------------------------------------ K1 / K2
def sgd_step(master, grad, mom, model, *, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
             first_step=False, grad_scale=1.0, dscale: Optional[torch.Tensor] = None):
    if _is_dev(master):
        _need_native("sgd_step").sgd_step(master, grad, mom, model, float(lr), float(momentum), float(dampening),
                                          float(weight_decay), bool(nesterov), bool(first_step), float(grad_scale),
                                          dscale)
    else:
        reference.sgd_step(master, grad, mom, model, lr=lr, momentum=momentum, dampening=dampening,
                           weight_decay=weight_decay, nesterov=nesterov, first_step=first_step,
                           grad_scale=grad_scale, dscale=dscale)


def adam_step(master, grad, m1, m2, model, *, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, adamw=True,
              step=1, grad_scale=1.0, dscale: Optional[torch.Tensor] = None):
    if _is_dev(master):
        _need_native("adam_step").adam_step(master, grad, m1, m2, model, float(lr), float(beta1), float(beta2),
                                            float(eps), float(weight_decay), bool(adamw), int(step),
                                            float(grad_scale), dscale)
    else:
        reference.adam_step(master, grad, m1, m2, model, lr=lr, beta1=beta1, beta2=beta2, eps=eps,
                            weight_decay=weight_decay, adamw=adamw, step=step, grad_scale=grad_scale, dscale=dscale)


def grad_norm(flats: Sequence[torch.Tensor], max_norm: float = 0.0, scale: float = 1.0) -> torch.Tensor:
    """[global L2 norm, clip coefficient] as a 2-element fp32 tensor on the flats' device (no host sync)."""
    if _is_dev(flats[0]):
        return _need_native("grad_norm").grad_norm(list(flats), float(max_norm), float(scale))
    return reference.grad_norm(flats, max_norm, scale)


# ---------------------------------------------------------------------- K3
class _NormFn(torch.autograd.Function):
    """K3 norm.  Modes: plain (y), residual (y = N(x + res), s = x + res) and fork
    (y = N(x), plus an alias of x for the block's residual path).  In residual and fork modes the
    second output's gradient is added inside the same backward pass (``dres``), so a tensor used
    both as the norm input and as the residual costs no separate autograd accumulation."""

    @staticmethod
    def forward(ctx, x, res, w, b, eps, rms, fork):
        shape = x.shape
        xc = x.contiguous()
        rc = res.contiguous() if res is not None else None
        y, s, mean, rstd = _need_native("norm_fwd").norm_fwd(xc, rc, w, b, float(eps), bool(rms))
        saved_x = s if res is not None else xc
        ctx.save_for_backward(saved_x, w, mean, rstd)
        # the input came straight from a biased madnn Linear (the transformer residual stream): the
        # backward also returns dx's column sums for that Linear's bias gradient (_LinearFn reads
        # them off the gradient tensor instead of running its own column-sum pass)
        ctx.colsum = NORM_COLSUM and _from_biased_linear(x)
        ctx.colsum_bf16 = ctx.colsum and _linear_bias_dtype(x) == torch.bfloat16
        ctx.rms = rms
        ctx.has_bias = b is not None
        ctx.has_res = res is not None
        ctx.fork = fork and res is None
        ctx.shape = shape
        if res is not None:
            return y.view(shape), s.view(shape)
        if ctx.fork:
            return y.view(shape), x.view_as(x)
        return y.view(shape), None

    @staticmethod
    def backward(ctx, dy, ds):
        x, w, mean, rstd = ctx.saved_tensors
        dres = ds.contiguous() if ((ctx.has_res or ctx.fork) and ds is not None) else None
        dx, dw, db, cs = torch.ops.madnn.norm_bwd(dy.contiguous(), x, w, mean, rstd, dres, ctx.rms, ctx.has_bias,
                                                  ctx.colsum, ctx.colsum_bf16)
        dx = dx.view(ctx.shape)
        if ctx.colsum:
            _attach(dx, "_madnn_colsum", cs)
        return dx, (dx if ctx.has_res else None), dw, (db if ctx.has_bias else None), None, None, None


NORM_COLSUM = os.environ.get("MADNN_NORM_COLSUM", "1") != "0"  # A/B switch (see _NormFn.forward)


_VIEW_NODES = ("ViewBackward0", "ReshapeAliasBackward0", "UnsafeViewBackward0")


def _linear_bias_dtype(x: torch.Tensor):
    """The bias dtype of the madnn Linear that produced ``x`` (directly or through one reshape), else
    None (no such Linear, or one without a bias)."""
    gf = x.grad_fn
    if gf is not None and type(gf).__name__ in _VIEW_NODES and len(gf.next_functions) == 1:
        gf = gf.next_functions[0][0]
    if gf is None or type(gf).__name__ not in ("_LinearFnBackward", "_GeluMLPFnBackward", "_LinearTeeFnBackward"):
        return None
    return getattr(gf, "bias_dtype", None)


def _from_biased_linear(x: torch.Tensor) -> bool:
    """``x`` is a biased madnn Linear's output, or one reshape of it (autograd passes the gradient
    back through the view, whose base then carries the consumer's column sums)."""
    return _linear_bias_dtype(x) is not None


def _norm(x, weight, bias, eps, rms, residual, fork=False):
    if _is_dev(x):
        if weight is None:
            raise ValueError("madnn norm kernels need an affine weight")
        y, s = _NormFn.apply(x, residual, weight, bias, eps, rms, fork)
        return (y, s) if (residual is not None or fork) else y
    y = reference.norm(x, weight, bias, eps, rms, residual)
    return (y, x) if (fork and residual is None) else y


def layer_norm(x, weight, bias=None, eps: float = 1e-5, residual: Optional[torch.Tensor] = None, fork: bool = False):
    """LayerNorm over the last dim.  With ``residual``: returns (LN(x + residual), x + residual).
    With ``fork``: returns (LN(x), x) where the second output's gradient is summed into x's
    inside the LN backward kernel (use it as the block's residual path)."""
    return _norm(x, weight, bias, eps, False, residual, fork)


def rms_norm(x, weight, eps: float = 1e-6, residual: Optional[torch.Tensor] = None, fork: bool = False):
    """RMSNorm over the last dim.  With ``residual``: returns (RMS(x + residual), x + residual);
    with ``fork``: (RMS(x), x) as in :func:`layer_norm`."""
    return _norm(x, weight, None, eps, True, residual, fork)


def _attach(t: torch.Tensor, name: str, value) -> None:
    """Side-channel a by-product (a column sum, a bit mask, BN partial sums) onto the gradient
    tensor ``t`` it describes, stamped with ``t``'s version counter: if autograd later accumulates
    another consumer's gradient into ``t`` in place, the stamp no longer matches."""
    setattr(t, name, (value, t._version))


def _attached(t: Optional[torch.Tensor], name: str, strict: bool = False):
    """The by-product :func:`_attach` put on ``t`` (or on the base ``t`` views), or None when
    there is none or ``t`` was modified since; ``strict`` raises instead for by-products whose
    absence changes the meaning of ``t`` (a deferred ReLU mask)."""
    if t is None:
        return None
    rec = getattr(t, name, None)
    if rec is None and t._base is not None and t.numel() == t._base.numel():
        rec = getattr(t._base, name, None)
    if rec is None:
        return None
    value, version = rec
    if t._version != version:
        if strict:
            raise RuntimeError(f"madnn: gradient carrying {name} was modified in place after it was produced "
                               "(a second consumer's gradient accumulated into it); disable the deferral "
                               "(MADNN_DEFER_RES_MASK=0) for this model")
        return None
    return value


# ---------------------------------------------------------------------- K5
class _BNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, nbt, training, momentum, eps, relu, stats):
        y, mean, invstd, scale, shift, mask = torch.ops.madnn.bn_fwd(x, residual, weight, bias, running_mean,
                                                                      running_var, nbt, bool(training),
                                                                      float(momentum), float(eps), bool(relu),
                                                                      stats if training else None)
        # the residual itself is not saved: with ReLU its only backward use (the mask) is the bit mask
        ctx.save_for_backward(x, mask, weight, mean, invstd, scale, shift)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.has_w = weight is not None
        # the residual is a ResNet block's identity whose only consumer is this BN and whose gradient
        # is summed inside a K9 data grad (Bottleneck marks it): hand that kernel dy and the ReLU bit
        # mask instead of writing the masked copy of dy (one activation-sized write less)
        ctx.defer = (DEFER_RES_MASK and relu and residual is not None and mask.numel() > 0
                     and getattr(residual, "_madnn_defer_mask", False))
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, mean, invstd, scale, shift = ctx.saved_tensors
        need_w = ctx.has_w and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        defer = ctx.defer and dy.dtype == x.dtype and dy.stride() == x.stride()
        dx, dw, db, dres = torch.ops.madnn.bn_bwd(dy, x, mask if mask.numel() else None, ctx.has_res, weight,
                                                  mean, invstd, scale, shift, ctx.relu, need_w, not defer)
        if defer:
            dres = dy.view_as(dy)
            _attach(dres, "_madnn_resmask", mask)
        return (dx, dw if need_w else None, db if need_w else None, dres if ctx.has_res else None,
                None, None, None, None, None, None, None, None)


DEFER_RES_MASK = os.environ.get("MADNN_DEFER_RES_MASK", "1") != "0"  # A/B switch (see _BNFn.forward)


def _apply_bit_mask(t: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """``t`` (NHWC / row-major) with the elements whose bit in ``mask`` (8 per byte, memory order) is
    clear set to zero -- the unfused fallback of a deferred ReLU-masked residual gradient."""
    flat = _nhwc(t).permute(0, 2, 3, 1).reshape(-1) if t.dim() == 4 else t.reshape(-1)
    shifts = torch.arange(8, device=mask.device, dtype=torch.uint8)
    keep = mask.reshape(-1, 1).bitwise_right_shift(shifts).bitwise_and(1).reshape(-1)
    out = (flat * keep.to(flat.dtype)).view(flat.shape)
    if t.dim() == 4:
        n, c, h, w = t.shape
        return out.view(n, h, w, c).permute(0, 3, 1, 2)
    return out.view(t.shape)


def bn_supported(x: torch.Tensor, weight: Optional[torch.Tensor]) -> bool:
    """Shapes/layouts the fused NHWC BatchNorm kernel handles."""
    if x.device.type != "cuda" or x.dtype not in (torch.bfloat16, torch.float32, torch.float16):
        return False
    c = x.size(1)
    if c % 8 or c > 2048:
        return False
    if weight is not None and weight.dtype != torch.float32:
        return False
    if x.dim() == 2:
        return x.is_contiguous()
    return x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)


def batch_norm_act(x, weight, bias, running_mean, running_var, num_batches_tracked=None, *, training: bool,
                   momentum: float = 0.1, eps: float = 1e-5, relu: bool = False,
                   residual: Optional[torch.Tensor] = None, stats: Optional[torch.Tensor] = None):
    """act(BN(x) + residual) for NHWC activations in one fused kernel per direction.

    Device tensors of a supported layout use the K5 HIP kernels (batch statistics,
    running-stat update and num_batches_tracked increment included); anything else
    (CPU, NCHW, unsupported C, eval-mode backward) uses the eager composition.
    ``stats``: per-channel partial (sum, sum of squares) of ``x`` already computed by the
    kernel that produced it (``conv1x1(..., stats=True)``); the statistics pass is skipped.
    """
    needs_grad = torch.is_grad_enabled() and (x.requires_grad or (weight is not None and weight.requires_grad)
                                              or (residual is not None and residual.requires_grad))
    fused = bn_supported(x, weight) and (training or not needs_grad) and momentum is not None
    if fused and residual is not None:
        fused = residual.dtype == x.dtype and residual.shape == x.shape and residual.stride() == x.stride()
    if fused:
        _need_native("batch_norm_act")
        return _BNFn.apply(x, weight, bias, residual, running_mean, running_var,
                           num_batches_tracked if training else None, training, momentum, eps, relu, stats)
    return reference.batch_norm_act(x, weight, bias, running_mean, running_var, num_batches_tracked,
                                    training=training, momentum=momentum, eps=eps, relu=relu, residual=residual)


class _BNDualFn(torch.autograd.Function):
    """relu(BN(x) + BN_r(r)), training.  The residual BatchNorm's output is never materialised:
    one apply pass forward, one reduction + one apply pass backward serve both BNs."""

    @staticmethod
    def forward(ctx, x, r, weight, bias, weight_r, bias_r, bn, bn_r, stats, stats_r):
        out = torch.ops.madnn.bn_fwd_dual(x, r, weight, bias, bn.running_mean, bn.running_var,
                                          bn.num_batches_tracked, float(bn.momentum), float(bn.eps), stats,
                                          weight_r, bias_r, bn_r.running_mean, bn_r.running_var,
                                          bn_r.num_batches_tracked, float(bn_r.momentum), float(bn_r.eps), stats_r)
        y, mask, mean, invstd, _, _, mean_r, invstd_r, _, _ = out
        ctx.save_for_backward(x, r, mask, weight, mean, invstd, weight_r, mean_r, invstd_r)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, r, mask, weight, mean, invstd, weight_r, mean_r, invstd_r = ctx.saved_tensors
        dx, dr, dw, db, dw_r, db_r = torch.ops.madnn.bn_bwd_dual(dy, x, r, mask, weight, mean, invstd,
                                                                 weight_r, mean_r, invstd_r)
        return dx, dr, dw, db, dw_r, db_r, None, None, None, None


def batch_norm_dual_supported(x: torch.Tensor, r: torch.Tensor, bn, bn_r) -> bool:
    """Shapes/modes :func:`batch_norm_add_bn_relu` runs as one fused kernel pair."""
    def ok(m):
        return (m.training and m.track_running_stats and m.affine and m.momentum is not None
                and m.weight.dtype == torch.float32)
    if not (isinstance(x, torch.Tensor) and isinstance(r, torch.Tensor)):   # e.g. fx tracing proxies
        return False
    return (x.dtype == torch.bfloat16 and bn_supported(x, bn.weight) and r.shape == x.shape
            and r.dtype == x.dtype and r.stride() == x.stride() and ok(bn) and ok(bn_r))


def batch_norm_add_bn_relu(x, r, bn, bn_r, stats=None, stats_r=None):
    """``relu(bn(x) + bn_r(r))`` for two training-mode BatchNorm modules (ResNet's bn3 plus the
    downsample path's BN): both BNs' statistics, running-stat updates and gradients, with the
    residual BN applied inside bn's passes instead of in passes of its own (K5 ``RAFF`` variants).
    Falls back to the two-module composition when the fused path does not apply."""
    if batch_norm_dual_supported(x, r, bn, bn_r):
        _need_native("batch_norm_add_bn_relu")
        return _BNDualFn.apply(x, r, bn.weight, bn.bias, bn_r.weight, bn_r.bias, bn, bn_r, stats, stats_r)
    idt = bn_r(r, stats=stats_r) if _is_fused_bn(bn_r) else bn_r(r)
    return bn(x, residual=idt, relu=True, stats=stats) if _is_fused_bn(bn) else torch.relu(bn(x) + idt)


def _is_fused_bn(m) -> bool:
    from ..nn.norm import FusedBatchNorm2d
    return isinstance(m, FusedBatchNorm2d)


# ---------------------------------------------------------------------- K7
class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, arg = torch.ops.madnn.maxpool_fwd(x, k, s, p, True)
        ctx.save_for_backward(arg)
        ctx.geom = (x.size(2), x.size(3), k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        return torch.ops.madnn.maxpool_bwd(dy, arg, *ctx.geom), None, None, None


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def max_pool_supported(x: torch.Tensor, kernel_size, stride=None, padding=0, dilation=1,
                       ceil_mode: bool = False) -> bool:
    """Layouts/geometries the K7 NHWC max-pool kernel handles."""
    k, s, p, d = _pair(kernel_size), _pair(stride if stride else kernel_size), _pair(padding), _pair(dilation)
    if x.device.type != "cuda" or x.dtype not in (torch.bfloat16, torch.float32, torch.float16):
        return False
    if x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last) or x.size(1) % 8:
        return False
    if k[0] != k[1] or s[0] != s[1] or p[0] != p[1] or d != (1, 1) or ceil_mode:
        return False
    return k[0] * k[0] <= 255 and 2 * p[0] <= k[0] and x.numel() < 2**31


def max_pool2d(x: torch.Tensor, kernel_size, stride=None, padding=0, dilation=1, ceil_mode: bool = False):
    """Square max-pooling; NHWC device tensors run the K7 kernels (argmax kept as one byte per
    output element, gather backward), everything else ``F.max_pool2d``."""
    if max_pool_supported(x, kernel_size, stride, padding, dilation, ceil_mode):
        _need_native("max_pool2d")
        k = _pair(kernel_size)[0]
        s = _pair(stride if stride else kernel_size)[0]
        p = _pair(padding)[0]
        if torch.is_grad_enabled() and x.requires_grad:
            return _MaxPoolFn.apply(x, k, s, p)
        return torch.ops.madnn.maxpool_fwd(x, k, s, p, False)[0]
    return torch.nn.functional.max_pool2d(x, kernel_size, stride, padding, dilation, ceil_mode)


# ---------------------------------------------------------------------- K6
class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, shift, vocab, ignore_index, scale):
        lg = logits.contiguous()
        tg = targets.contiguous()
        used = tg[:, 1:] if shift else tg
        # the loss is ``scale`` x the mean: a microbatch's 1 / M folded in here reaches the fused
        # gradient at forward time, so its backward sees an upstream gradient of exactly 1 and the
        # rescale pass over the logit gradient exits at once (at 32 x 1024 tokens per microbatch that
        # pass was 1.3 ms of GPT-2 medium's LM head, profiles/r6_gpt2m_mb32_steady_steps.md)
        cnt = ((used != ignore_index) & (used >= 0) & (used < vocab)).sum().clamp(min=1).to(torch.float32) / scale
        ctx.grad = None
        ctx.fused = bool(ctx.needs_input_grad[0] and XENT_FUSED and _xent_fused_ok(lg))
        if ctx.fused:
            # K6f: the gradient is finished here, in the same pass over the logits as the loss
            # (backward only applies the upstream scale, a no-op launch for loss.backward())
            loss_rows, ctx.grad = torch.ops.madnn.xent_fused(lg, tg, bool(shift), int(vocab), int(ignore_index),
                                                            (1.0 / cnt).reshape(1))
            return loss_rows.sum() / cnt
        loss_rows, lse = torch.ops.madnn.xent_fwd(lg, tg, bool(shift), int(vocab), int(ignore_index))
        ctx.save_for_backward(lg, tg, lse, cnt)
        ctx.shift, ctx.vocab, ctx.ignore_index = shift, vocab, ignore_index
        return loss_rows.sum() / cnt

    @staticmethod
    def backward(ctx, g):
        if ctx.fused:
            grad, ctx.grad = ctx.grad, None
            if grad is None:
                raise RuntimeError("madnn cross_entropy: the fused (K6f) gradient was already consumed by an "
                                   "earlier backward; set MADNN_XENT_FUSED=0 to backward through it twice")
            torch.ops.madnn.xent_rescale(grad, g.to(torch.float32).reshape(1))
            return grad, None, None, None, None, None
        lg, tg, lse, cnt = ctx.saved_tensors
        gscale = (g.to(torch.float32) / cnt).reshape(1)
        grad = torch.ops.madnn.xent_bwd(lg, tg, lse, ctx.shift, ctx.vocab, ctx.ignore_index, gscale)
        return grad, None, None, None, None, None


XENT_FUSED = os.environ.get("MADNN_XENT_FUSED", "1") != "0"  # A/B switch


def _xent_fused_ok(lg: torch.Tensor) -> bool:
    """K6f preconditions (mirrored by xent_fused_ok in binding.cpp): 16-bit contiguous logits whose rows
    are 16-byte aligned and fit 32 chunks of 8 per lane of a 512-lane workgroup."""
    ld = lg.size(-1)
    return (lg.dtype in (torch.bfloat16, torch.float16) and lg.is_contiguous() and ld % 8 == 0
            and ld // 8 <= 32 * 512 and lg.data_ptr() % 16 == 0)


def cross_entropy(logits: torch.Tensor, targets: torch.Tensor, *, shift: bool = False, vocab: Optional[int] = None,
                  ignore_index: int = -100, scale: float = 1.0) -> torch.Tensor:
    """Mean token cross entropy of ``logits[..., :vocab]`` (fp32 math, one fused kernel each way),
    times ``scale`` (a microbatched step's 1 / M, applied inside the kernels: see _XentFn).

    ``shift=True`` is the causal-LM form: logits[:, t] predicts targets[:, t+1] and the
    last position carries no loss — no slicing copies of the logit matrix are made.
    Columns >= ``vocab`` (a padded vocabulary) are excluded from the softmax."""
    v = vocab or logits.size(-1)
    if _is_dev(logits) and logits.dtype in (torch.bfloat16, torch.float32, torch.float16):
        _need_native("cross_entropy")
        return _XentFn.apply(logits, targets, shift, v, ignore_index, float(scale))
    out = reference.cross_entropy(logits, targets, shift=shift, vocab=v, ignore_index=ignore_index)
    return out * scale if scale != 1.0 else out


def scaled_loss(fn, out, targets, scale: float):
    """``fn(out, targets) * scale`` -- with the scale passed INTO ``fn`` when it takes one (madnn's
    model losses: the cross entropy folds it into its fused gradient), else applied after."""
    import inspect

    try:
        takes = "scale" in inspect.signature(fn).parameters
    except (TypeError, ValueError):
        takes = False
    if takes and scale != 1.0:
        return fn(out, targets, scale=scale)
    loss = fn(out, targets)
    return loss * scale if scale != 1.0 else loss


# ---------------------------------------------------------------------- K8
class _AttnFn(torch.autograd.Function):
    """q [B,S,H,D], k/v [B,S,Hkv,D] (strided views) -> o [B,S,H,D] contiguous."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        o, lse = torch.ops.madnn.attn_fwd(q, k, v, bool(causal), float(scale))
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        torch.ops.madnn.attn_bwd(do, q, k, v, o, lse, dq, dk, dv, ctx.causal, float(ctx.scale))
        return dq, dk, dv, None, None


class _AttnPackedFn(torch.autograd.Function):
    """qkv [B,S,H+2*Hkv,D] (one projection's output) -> o [B,S,H,D]; dQKV is written in place
    into one buffer (no split/cat copies in either direction)."""

    @staticmethod
    def forward(ctx, qkv, heads, kv_heads, causal, scale):
        q, k, v = qkv.split([heads, kv_heads, kv_heads], dim=2)
        o, lse = torch.ops.madnn.attn_fwd(q, k, v, bool(causal), float(scale))
        ctx.save_for_backward(qkv, o, lse)
        ctx.meta = (heads, kv_heads, bool(causal), float(scale))
        # qkv is (a view of) a biased madnn Linear's output: the backward kernels also sum dQKV's
        # columns, which that Linear takes as its bias gradient (no column-sum pass of its own)
        ctx.colsum = ATTN_COLSUM and _from_biased_linear(qkv)
        ctx.colsum_dtype = torch.bfloat16 if ctx.colsum and _linear_bias_dtype(qkv) == torch.bfloat16 else torch.float32
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        heads, kv_heads, causal, scale = ctx.meta
        q, k, v = qkv.split([heads, kv_heads, kv_heads], dim=2)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv.split([heads, kv_heads, kv_heads], dim=2)
        cs = None
        if ctx.colsum:
            cs = torch.empty((heads + 2 * kv_heads) * qkv.size(-1), dtype=ctx.colsum_dtype, device=qkv.device)
        torch.ops.madnn.attn_bwd(do, q, k, v, o, lse, dq, dk, dv, causal, scale, cs)
        if cs is not None:
            _attach(dqkv, "_madnn_colsum", cs)
        return dqkv, None, None, None, None


ATTN_COLSUM = os.environ.get("MADNN_ATTN_COLSUM", "1") != "0"  # A/B switch (see _AttnPackedFn.forward)


def attention_supported(t: torch.Tensor, head_dim: int, dropout: float = 0.0) -> bool:
    """Inputs the K8 attention kernels take: bf16 HIP tensors, head dim 64/128, no dropout."""
    return (t.device.type == "cuda" and t.dtype == torch.bfloat16 and head_dim in (64, 128)
            and dropout == 0.0 and t.stride(-1) == 1)


def attention(q, k, v, *, causal: bool = True, scale: Optional[float] = None):
    """Scaled-dot-product attention on [B, S, heads, D] tensors (GQA when k/v have fewer heads).
    Returns [B, S, H, D].  HIP bf16 inputs run K8; anything else runs SDPA."""
    scale = scale if scale is not None else q.size(-1) ** -0.5
    if attention_supported(q, q.size(-1)):
        _need_native("attention")
        return _AttnFn.apply(q, k, v, causal, scale)
    return reference.attention(q, k, v, causal=causal, scale=scale)


def attention_qkvpacked(qkv, heads: int, kv_heads: int, *, causal: bool = True, scale: Optional[float] = None):
    """Attention straight from a packed projection ``qkv`` [B, S, heads + 2*kv_heads, D]."""
    d = qkv.size(-1)
    scale = scale if scale is not None else d ** -0.5
    if attention_supported(qkv, d) and qkv.is_contiguous():
        _need_native("attention")
        return _AttnPackedFn.apply(qkv, heads, kv_heads, causal, scale)
    q, k, v = qkv.split([heads, kv_heads, kv_heads], dim=2)
    return reference.attention(q, k, v, causal=causal, scale=scale)


# ---------------------------------------------------------------- K14 / K15
def _rope_rotate(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, inverse: bool) -> torch.Tensor:
    """Eager reference of K14 on [B, S, heads, D] (fp32 math): (a, b) -> (a c -+ b s, b c +- a s)."""
    d = x.size(-1) // 2
    c, sn = cos[: x.size(1), None, :d].float(), sin[: x.size(1), None, :d].float()
    a, b = x[..., :d].float(), x[..., d:].float()
    if inverse:
        return torch.cat([a * c + b * sn, b * c - a * sn], -1).to(x.dtype)
    return torch.cat([a * c - b * sn, b * c + a * sn], -1).to(x.dtype)


class _RopeQKVFn(torch.autograd.Function):
    """RoPE on the q and k heads of a packed QKV projection (K14): one pass writes a new packed
    tensor (q, k rotated, v copied) that the attention reads in place; the backward applies the
    transpose rotation in place on the incoming dQKV (the attention backward's own fresh output,
    consumed only here), so the packed gradient flows on to the projection with no copy."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, rot_heads):
        ctx.save_for_backward(cos, sin)
        ctx.rot = rot_heads
        if _is_dev(qkv):
            return torch.ops.madnn.rope_qkv(qkv, cos, sin, rot_heads, False)
        out = qkv.clone()
        out[:, :, :rot_heads] = _rope_rotate(qkv[:, :, :rot_heads], cos, sin, False)
        return out

    @staticmethod
    def backward(ctx, g):
        cos, sin = ctx.saved_tensors
        g = g.contiguous()
        if _is_dev(g):
            torch.ops.madnn.rope_qkv_(g, cos, sin, ctx.rot, True)
        else:
            g = g.clone()
            g[:, :, : ctx.rot] = _rope_rotate(g[:, :, : ctx.rot], cos, sin, True)
        return g, None, None, None


def rope_qkv(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, rot_heads: int) -> torch.Tensor:
    """``qkv`` [B, S, heads, D] with heads ``0..rot_heads-1`` (q then k) rotated by the RoPE tables
    ``cos`` / ``sin`` (fp32 [>= S, D], halves duplicated), as a new packed tensor.  HIP bf16
    contiguous inputs run K14 (``madnn/ops/csrc/glue.hip``); others the eager reference."""
    if _is_dev(qkv):
        _need_native("rope_qkv")
        if not (qkv.dtype == torch.bfloat16 and qkv.is_contiguous() and qkv.size(-1) % 16 == 0
                and cos.dtype == torch.float32 and cos.is_contiguous()):
            raise ValueError("rope_qkv: needs a contiguous bf16 qkv (D % 16 == 0) and fp32 tables")
        if qkv.data_ptr() % 16:
            qkv = qkv.clone()   # a slice off a 16-byte boundary: K14 moves 16 B per lane
        if cos.data_ptr() % 16 or sin.data_ptr() % 16:
            cos, sin = cos.clone(), sin.clone()
    return _RopeQKVFn.apply(qkv, cos, sin, rot_heads)


class _SwiGLUFn(torch.autograd.Function):
    """h = silu(g) * u from the fused gate_up output [..., 2I] (K15); the backward writes the packed
    d[g | u] the gate_up Linear consumes (no split / cat)."""

    @staticmethod
    def forward(ctx, gu):
        ctx.save_for_backward(gu)
        return torch.ops.madnn.swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dh):
        (gu,) = ctx.saved_tensors
        if dh.data_ptr() % 16 or not dh.is_contiguous():
            dh = dh.contiguous().clone()   # K15 moves 16 B per lane: a fresh (aligned) buffer
        return torch.ops.madnn.swiglu_bwd(dh, gu)


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    """``silu(g) * u`` with ``g, u = gu.chunk(2, -1)``: K15 on contiguous HIP bf16, eager otherwise."""
    if (_is_dev(gu) and gu.dtype == torch.bfloat16 and gu.is_contiguous() and gu.size(-1) % 16 == 0
            and gu.data_ptr() % 16 == 0):
        _need_native("swiglu")
        return _SwiGLUFn.apply(gu)
    g, u = gu.chunk(2, dim=-1)
    return F.silu(g) * u


# ---------------------------------------------------------------------- K9
def _nhwc(t: torch.Tensor) -> torch.Tensor:
    return t.contiguous(memory_format=torch.channels_last) if t.dim() == 4 else t.contiguous()


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[M, C] view of an NHWC (or 2-D) tensor."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.size(1)) if t.dim() == 4 else t


def conv1x1_route(cin: int, cout: int) -> tuple:
    """Which implementation runs each pass of a stride-1 1x1 conv, from the per-shape A/B of
    ResNet-50's convolutions on MI355X (round-1 A/B drivers, now in git history;
    profiles/r1_k9_conv1x1_ab.json):

    * forward: K9 (+ the BatchNorm statistics in its epilogue) where it is at least as fast as
      MIOpen once the BN statistics pass it removes is counted -- the HBM-bound shapes
      (Cin <= 256, or an expanding Cout >= 2 Cin); MIOpen on the deep contracting reductions;
    * data grad: K9 on the HBM-bound shapes (Cin <= 256 and Cout <= 512), hipBLASLt GEMM on the
      deep ones; both add the identity path's gradient in the epilogue / with beta = 1;
    * weight grad: per shape the fastest of MIOpen, K12 split-K and K9 split-M (timed once,
      :func:`tuned_wgrad`; K9's slabs are reduced and cast to bf16 in one pass, no zero fill).
    Same-box full-step A/B of these choices: docs/PERF.md ("K9 routing").
    ``MADNN_K9_DGRAD=wide`` / ``MADNN_K9_WGRAD=k9`` select the alternatives.
    """
    fwd = "k9" if (cin <= 256 or cout >= 2 * cin) else "miopen"
    if _K9_DGRAD == "narrow":
        dgrad = "k9" if (cin <= 256 and cout <= 512) else "gemm"
    else:
        dgrad = "gemm" if (cout >= 1024 and cout >= 4 * cin) else "k9"
    return fwd, dgrad, _K9_WGRAD


_K9_WGRAD = os.environ.get("MADNN_K9_WGRAD", "miopen")  # "k9" | "miopen" (A/B runs)
_K9_DGRAD = os.environ.get("MADNN_K9_DGRAD", "narrow")  # "wide" | "narrow" (A/B runs)


class _Conv1x1Fn(torch.autograd.Function):
    """Stride-1 1x1 convolution on NHWC bf16 (see :func:`conv1x1_route`).  With ``fork`` the
    input is also returned (as the block's identity path); its gradient is then accumulated
    inside the data-grad kernel instead of by a separate autograd add.  ``fork == 2`` returns the
    stride-2 subsample ``x[:, :, ::2, ::2]`` instead (compact NHWC: the input of a ResNet
    downsample convolution, which then runs as a stride-1 1x1 on a quarter of the pixels); its
    compact gradient is added into the even pixels of this convolution's data grad -- no
    zero-filled full-resolution gradient and no stride-2 data-grad kernel."""

    @staticmethod
    def forward(ctx, x, w, stats, fork):
        fwd, dgrad, wgrad = conv1x1_route(x.size(1), w.size(0))
        if fwd == "k9":
            y, part = torch.ops.madnn.conv1x1_fwd(x, w, bool(stats))
        else:
            y = torch.nn.functional.conv2d(x, w) if x.dim() == 4 else torch.mm(x, w.reshape(w.size(0), -1).t())
            part = x.new_empty((0, 2, w.size(0)), dtype=torch.float32)
        ctx.save_for_backward(x, w)
        ctx.route = (dgrad, wgrad)
        ctx.fork = fork
        ctx.mark_non_differentiable(part)
        if fork == 2:
            return y, part, x[:, :, ::2, ::2].contiguous(memory_format=torch.channels_last)
        if fork:
            return y, part, x.view_as(x)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart, dfork=None):
        x, w = ctx.saved_tensors
        dgrad, wgrad = ctx.route
        dy = _nhwc(dy.to(x.dtype))
        sub = None
        if ctx.fork == 2:
            sub, dfork = dfork, None
        # a deferred ReLU mask (_BNFn): the identity gradient is dfork where its bit is set
        resmask = _attached(dfork, "_madnn_resmask", strict=True)
        res = _nhwc(dfork.to(x.dtype)) if dfork is not None else None
        if resmask is not None and not (ctx.needs_input_grad[0] and dgrad == "k9"):
            res, resmask = _apply_bit_mask(res, resmask), None
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if dgrad == "k9":
                dx = torch.ops.madnn.conv1x1_dgrad(dy, w, res, resmask)
            else:
                w2 = w.reshape(w.size(0), -1)
                if res is not None:
                    # beta = 1 GEMM accumulating straight into the identity path's gradient buffer
                    # (addmm with out= would first copy it); res is this backward's own tensor
                    dx = res if res._base is None else _nhwc(res.clone())
                    _rows(dx).addmm_(_rows(dy), w2)
                else:
                    dx = torch.empty_like(x)
                    torch.mm(_rows(dy), w2, out=_rows(dx))
        elif res is not None:
            dx = res
        if sub is not None:
            if dx is None:
                dx = torch.zeros_like(x)
            dx[:, :, ::2, ::2].add_(sub.to(dx.dtype))
        if ctx.needs_input_grad[1]:
            if wgrad == "k9":
                dw = _k9_wgrad(dy, x, w)
            else:
                dw = _conv1x1_wgrad_lib(dy, x, w)
        return dx, dw, None, None


def conv1x1_supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Inputs the K9 path takes: bf16 HIP tensors, NHWC (or 2-D [M, C]), channels % 64 == 0."""
    if x.device.type != "cuda" or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or x.numel() == 0:
        return False
    if x.dim() == 4:
        if not x.is_contiguous(memory_format=torch.channels_last):
            return False
    elif x.dim() != 2 or not x.is_contiguous():
        return False
    cin, cout = x.size(1), w.size(0)
    if w.numel() != cin * cout or w.stride(0) != cin or w.stride(1) != 1:
        return False
    return cin % 64 == 0 and cout % 64 == 0


def conv1x1(x: torch.Tensor, w: torch.Tensor, *, stats: bool = False, fork: bool = False):
    """Stride-1 1x1 convolution ``x (*) w`` of an NHWC bf16 HIP tensor (K9 / library per pass,
    :func:`conv1x1_route`).  ``stats``: also return the per-workgroup channel sums / sums of
    squares of y for :func:`batch_norm_act` (None when the forward did not run on K9).
    ``fork``: also return an alias of ``x`` to use as the residual path, whose gradient is then
    added inside this convolution's data-grad kernel; ``fork=2``: return the compact stride-2
    subsample of ``x`` instead (see :class:`_Conv1x1Fn`)."""
    _need_native("conv1x1")
    outs = _Conv1x1Fn.apply(x, w, stats, fork)
    y, part = outs[0], outs[1]
    ret = [y]
    if stats:
        ret.append(part if part.numel() else None)
    if fork:
        ret.append(outs[2])
    return ret[0] if len(ret) == 1 else tuple(ret)


class _BNReluConv1x1EpiFn(torch.autograd.Function):
    """``conv1x1(relu(bn(y)), w)`` in training with bn's backward reduction taken in the K9 data
    grad's epilogue (the conv3 shapes whose data grad runs on K9): forward = K5 apply + K9 with the
    output statistics; backward = K9 data grad (+ bn's sums), the routed weight grad on the stored
    activation, and bn's backward as finalize + apply only."""

    @staticmethod
    def forward(ctx, y, w, bn_w, bn_b, bn, stats_in, want_stats):
        a, mean, invstd, scale, shift, _ = torch.ops.madnn.bn_fwd(y, None, bn_w, bn_b, bn.running_mean,
                                                                  bn.running_var, bn.num_batches_tracked, True,
                                                                  float(bn.momentum), float(bn.eps), True, stats_in)
        fwd, _, wgrad = conv1x1_route(a.size(1), w.size(0))
        if fwd == "k9":
            out, part = torch.ops.madnn.conv1x1_fwd(a, w, bool(want_stats))
        else:
            out = torch.nn.functional.conv2d(a, w) if a.dim() == 4 else torch.mm(a, w.reshape(w.size(0), -1).t())
            part = a.new_empty((0, 2, w.size(0)), dtype=torch.float32)
        ctx.save_for_backward(y, a, w, bn_w, mean, invstd, scale, shift)
        ctx.wgrad = wgrad
        ctx.mark_non_differentiable(part)
        return out, part

    @staticmethod
    def backward(ctx, dout, _dpart):
        y, a, w, bn_w, mean, invstd, scale, shift = ctx.saved_tensors
        dout = _nhwc(dout.to(y.dtype))
        da, part = torch.ops.madnn.conv1x1_dgrad_bnb(dout, w, y, scale, shift)
        if ctx.wgrad == "k9":
            dw = _k9_wgrad(dout, a, w)
        else:
            dw = _conv1x1_wgrad_lib(dout, a, w)
        dy, dbw, dbb = torch.ops.madnn.bn_bwd_ext(da, y, bn_w, mean, invstd, scale, shift, part, True)
        need_bn = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        return dy, dw, dbw if need_bn else None, dbb if need_bn else None, None, None, None


def bn_relu_conv1x1(y: torch.Tensor, bn, w: torch.Tensor, *, stats_in: Optional[torch.Tensor] = None,
                    stats: bool = False):
    """``conv1x1(relu(bn(y)), w)`` (ResNet's bn2 -> conv3): when the data grad runs on K9, bn's
    backward reduction is taken in that kernel's epilogue.  ``stats_in``: ``y``'s partial
    statistics from its producer; ``stats``: also return the output's partial statistics (None if
    not computed).  (A BatchNorm-apply prologue inside K9's operand load lost its A/B --
    profiles/r2_ab_bn_prologue.json -- and was removed in round 6.)"""
    if bn_relu_conv1x1_epi_supported(y, bn, w):
        _need_native("bn_relu_conv1x1")
        out, part = _BNReluConv1x1EpiFn.apply(y, w, bn.weight, bn.bias, bn, stats_in, stats)
        return (out, part if part.numel() else None) if stats else out
    a = bn(y, relu=True, stats=stats_in) if _is_fused_bn(bn) else torch.relu(bn(y))
    if conv1x1_supported(a, w):
        return conv1x1(a, w, stats=stats)
    out = torch.nn.functional.conv2d(a, w.view(w.size(0), -1, 1, 1)) if a.dim() == 4 else torch.mm(
        a, w.reshape(w.size(0), -1).t())
    return (out, None) if stats else out


def bn_relu_conv1x1_epi_supported(y: torch.Tensor, bn, w: torch.Tensor) -> bool:
    """The data-grad-epilogue variant of :func:`bn_relu_conv1x1`: training BN (running stats, fp32
    affine) in front of a 1x1 convolution whose data grad routes to K9."""
    return (_BN_DGRAD_EPI and isinstance(y, torch.Tensor) and bn.training and bn.track_running_stats
            and bn.affine and bn.momentum is not None and bn.weight.dtype == torch.float32
            and conv1x1_supported(y, w) and bn_supported(y, bn.weight)
            and conv1x1_route(y.size(1), w.size(0))[1] == "k9")


class _BNReluMaxPoolFn(torch.autograd.Function):
    """``max_pool2d(relu(bn(y)), 3, 2, 1)`` in training (ResNet's stem): the BN apply + ReLU run
    inside the pool's window loads; backward gathers the pool gradient per input pixel inside the
    BN backward's two passes, so neither relu(bn(y)) nor its gradient is ever written to HBM."""

    @staticmethod
    def forward(ctx, y, bn_w, bn_b, bn, stats_in, p):
        mean, invstd, scale, shift = torch.ops.madnn.bn_coef(y, bn_w, bn_b, bn.running_mean, bn.running_var,
                                                             bn.num_batches_tracked, float(bn.momentum),
                                                             float(bn.eps), stats_in)
        out, arg = torch.ops.madnn.pool_bn_fwd(y, scale, shift, int(p))
        ctx.save_for_backward(y, arg, bn_w, mean, invstd, scale, shift)
        ctx.p = int(p)
        return out

    @staticmethod
    def backward(ctx, dp):
        y, arg, bn_w, mean, invstd, scale, shift = ctx.saved_tensors
        dy, dw, db = torch.ops.madnn.pool_bn_bwd(dp, arg, y, bn_w, mean, invstd, scale, shift, ctx.p)
        return dy, dw, db, None, None, None


def bn_relu_maxpool_supported(y: torch.Tensor, bn, pool) -> bool:
    """The stem shape the fused BN + ReLU + 3x3/s2 max-pool takes (training BN, bf16 NHWC)."""
    def pair(v):
        return tuple(v) if isinstance(v, (tuple, list)) else (v, v)
    return (_POOL_BN and isinstance(y, torch.Tensor) and y.device.type == "cuda" and y.dtype == torch.bfloat16 and y.dim() == 4
            and y.is_contiguous(memory_format=torch.channels_last) and bn.training and bn.track_running_stats
            and bn.affine and bn.momentum is not None and bn.weight.dtype == torch.float32
            and pair(pool.kernel_size) == (3, 3) and pair(pool.stride) == (2, 2) and pair(pool.padding) in ((1, 1), (0, 0))
            and pair(pool.dilation) == (1, 1) and not pool.ceil_mode and not pool.return_indices
            and y.size(1) % 8 == 0 and 256 % (y.size(1) // 8) == 0 and y.numel() < 2 ** 31)


def bn_relu_maxpool(y: torch.Tensor, bn, pool, stats_in: Optional[torch.Tensor] = None):
    """``pool(relu(bn(y)))`` with the BN apply fused into the pool (forward) and the pool gradient
    gathered inside the BN backward (:class:`_BNReluMaxPoolFn`); composition otherwise."""
    if bn_relu_maxpool_supported(y, bn, pool):
        _need_native("bn_relu_maxpool")
        p = pool.padding if isinstance(pool.padding, int) else pool.padding[0]
        return _BNReluMaxPoolFn.apply(y, bn.weight, bn.bias, bn, stats_in, p)
    a = bn(y, relu=True, stats=stats_in) if _is_fused_bn(bn) else torch.relu(bn(y))
    return pool(a)


# A/B knob: the stem's BN + ReLU + max-pool as one fused pair of passes (1) or as K5 + K7 (0)
_POOL_BN = os.environ.get("MADNN_POOL_BN", "1") != "0"


# ---------------------------------------------------------------------- K13
_K13 = os.environ.get("MADNN_CONV3X3", "1") != "0"
# weight grad: "auto" = K13 or MIOpen per shape, timed once (_conv3x3_wgrad); "k13" | "miopen" force one
_K13_WGRAD = os.environ.get("MADNN_CONV3X3_WGRAD", "auto")


def _k13_halo_ok(W: int) -> bool:
    # conv3.hip conv3x3_lds: halo pixels (rounded to whole 1-KiB DMA pieces) x 2*CH bytes + zero row +
    # two weight slots, at least the 32 KiB epilogue tile, must leave two workgroups per CU
    rb = 2 * 32   # 32 input channels per LDS stage (conv3.hip k13_ch)
    rpi = 1024 // rb
    cap = ((255 // W) * W + 4 * W + rpi - 1) // rpi * rpi
    return max(cap * rb + rb + 2 * 64 * rb, 32 * 1024) <= 80 * 1024


def conv3x3_supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Inputs K13 takes: NHWC bf16 HIP activations, bf16 [Co, Ci, 3, 3] weight, Ci and Co multiples
    of 64, image width whose input halo fits the kernel's LDS budget (W <= 56 or so)."""
    if not _K13 or x.device.type != "cuda" or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    if x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last) or x.numel() == 0:
        return False
    if w.dim() != 4 or tuple(w.shape[1:]) != (x.size(1), 3, 3):
        return False
    return x.size(1) % 64 == 0 and w.size(0) % 64 == 0 and _k13_halo_ok(x.size(3))


def _cl(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous(memory_format=torch.channels_last) else t.contiguous(memory_format=torch.channels_last)


def _conv3x3_wgrad(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """The 3x3 / stride-1 weight gradient on K13 (split over the pixels, fp32 slabs + one reduce) or
    MIOpen, whichever was faster for the shape (timed once, :func:`tuned_wgrad`).  At batch 2048 K13
    wins on the 56 / 28 / 14 maps and MIOpen on the 7x7 one (profiles/r3_resnet_wgrad_shapes_b2048.json);
    ``MADNN_CONV3X3_WGRAD=k13`` / ``miopen`` pin one."""
    k13 = lambda: torch.ops.madnn.conv3x3_wgrad(dy, x, w.dtype == torch.bfloat16)  # noqa: E731
    lib = lambda: torch.ops.aten.convolution_backward(  # noqa: E731
        dy, x, w, None, (1, 1), (1, 1), (1, 1), False, (0, 0), 1, (False, True, False))[1]
    if _K13_WGRAD == "k13":
        dw = k13()
    elif _K13_WGRAD == "miopen" or (_K13_WGRAD == "wide" and x.size(3) < 48):  # "wide": the round-2 rule
        dw = lib()
    elif _K13_WGRAD == "wide":
        dw = k13()
    else:
        dw = tuned_wgrad(("conv3x3",) + tuple(x.shape) + (w.size(0),), lib, k13)
    if dw.stride() != w.stride() or dw.dtype != w.dtype:
        dw = torch.empty_like(w).copy_(dw)
    return dw


class _Conv3x3Fn(torch.autograd.Function):
    """3x3 / stride 1 / pad 1 convolution (K13): MFMA implicit GEMM forward over an LDS-staged input
    halo with the BatchNorm statistics in its epilogue; the data gradient is the same kernel on the
    flipped, transposed weight (a correlation with W'[ci][kh][kw][co] = W[co][2-kh][2-kw][ci]); the
    weight gradient stays on MIOpen."""

    @staticmethod
    def forward(ctx, x, w, stats):
        y, part = torch.ops.madnn.conv3x3_fwd(x, _cl(w), bool(stats))
        ctx.save_for_backward(x, w)
        ctx.mark_non_differentiable(part)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        x, w = ctx.saved_tensors
        dy = _nhwc(dy.to(x.dtype))
        dx = dw = None
        if ctx.needs_input_grad[0]:
            wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
            dx = torch.ops.madnn.conv3x3_fwd(dy, wt, False)[0]
        if ctx.needs_input_grad[1]:
            dw = _conv3x3_wgrad(dy, x, w)
        return dx, dw, None


class _BNReluConv3x3Fn(torch.autograd.Function):
    """``conv3x3(relu(bn(y)), w)`` in training (ResNet's bn1 -> conv2).  Forward: the K5 BN apply
    (statistics from y's producer) and K13 with the output statistics.  Backward: K13's data grad
    also takes bn's backward sums over (d relu(bn(y)), y) in its epilogue, so the BN backward is
    finalize + apply only -- its reduction pass over two activation-sized tensors disappears."""

    @staticmethod
    def forward(ctx, y, w, bn_w, bn_b, bn, stats_in, want_stats):
        a, mean, invstd, scale, shift, _ = torch.ops.madnn.bn_fwd(y, None, bn_w, bn_b, bn.running_mean,
                                                                  bn.running_var, bn.num_batches_tracked, True,
                                                                  float(bn.momentum), float(bn.eps), True, stats_in)
        out, part = torch.ops.madnn.conv3x3_fwd(a, _cl(w), bool(want_stats))
        ctx.save_for_backward(y, a, w, bn_w, mean, invstd, scale, shift)
        ctx.mark_non_differentiable(part)
        return out, part

    @staticmethod
    def backward(ctx, dout, _dpart):
        y, a, w, bn_w, mean, invstd, scale, shift = ctx.saved_tensors
        dout = _nhwc(dout.to(y.dtype))
        wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
        da, part = torch.ops.madnn.conv3x3_fwd_bnb(dout, wt, y, scale, shift)
        dw = _conv3x3_wgrad(dout, a, w)
        dy, dbw, dbb = torch.ops.madnn.bn_bwd_ext(da, y, bn_w, mean, invstd, scale, shift, part, True)
        need_bn = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        return dy, dw, dbw if need_bn else None, dbb if need_bn else None, None, None, None


def bn_relu_conv3x3_supported(y: torch.Tensor, bn, w: torch.Tensor) -> bool:
    """Whether :func:`bn_relu_conv3x3` runs fused: training-mode BN with running statistics and an
    fp32 affine in front of a K13-shaped convolution whose data grad runs on K13."""
    return (_BN_DGRAD_EPI and isinstance(y, torch.Tensor) and bn.training
            and bn.track_running_stats and bn.affine and bn.momentum is not None
            and bn.weight.dtype == torch.float32 and conv3x3_supported(y, w) and y.size(1) == w.size(1)
            and bn_supported(y, bn.weight))


def bn_relu_conv3x3(y: torch.Tensor, bn, w: torch.Tensor, *, stats_in: Optional[torch.Tensor] = None,
                    stats: bool = False):
    """``conv3x3(relu(bn(y)), w)`` with bn's backward reduction taken in K13's data-grad epilogue
    (:class:`_BNReluConv3x3Fn`); composition of the two modules' paths otherwise."""
    if bn_relu_conv3x3_supported(y, bn, w):
        _need_native("bn_relu_conv3x3")
        out, part = _BNReluConv3x3Fn.apply(y, w, bn.weight, bn.bias, bn, stats_in, stats)
        return (out, part if part.numel() else None) if stats else out
    a = bn(y, relu=True, stats=stats_in) if _is_fused_bn(bn) else torch.relu(bn(y))
    if conv3x3_supported(a, w):
        return conv3x3(a, w, stats=stats)
    out = torch.nn.functional.conv2d(a, w, padding=1)
    return (out, None) if stats else out


# A/B knob: bn1's backward reduction in conv2's (K13) data-grad epilogue (1) or its own pass (0)
_BN_DGRAD_EPI = os.environ.get("MADNN_BN_DGRAD_EPI", "1") != "0"


def conv3x3(x: torch.Tensor, w: torch.Tensor, *, stats: bool = False):
    """``conv2d(x, w, stride=1, padding=1)`` of an NHWC bf16 HIP tensor on K13 (see
    :func:`conv3x3_supported`).  ``stats``: also return per-tile channel (sum, sum of squares)
    partials of y for :func:`batch_norm_act`."""
    _need_native("conv3x3")
    y, part = _Conv3x3Fn.apply(x, w, stats)
    return (y, part) if stats else y


# K13 at stride 2 (forward with the BN statistics; data / weight gradients on the library): taken up
# to this input width.  bench/conv3x3_s2_ab.py at ResNet-50's shapes (profiles/r5_conv3x3_s2_ab.json):
# K13 822 vs 834 us at 14 -> 7 (b2048; 222 vs 241 at b512) and the library needs a statistics pass
# besides; at 28 -> 14 and 56 -> 28 the taller stride-2 halo leaves K13 one or two workgroups per CU
# and MIOpen / CK run 38-43 % faster.
_K13_S2_MAX_W = int(os.environ.get("MADNN_CONV3X3_S2_MAX_W", "16"))


def conv3x3_s2_supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    """The stride-2 / pad-1 3x3 inputs K13 takes (even H and W up to ``MADNN_CONV3X3_S2_MAX_W``)."""
    if not _K13 or x.device.type != "cuda" or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    if x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last) or x.numel() == 0:
        return False
    if w.dim() != 4 or tuple(w.shape[1:]) != (x.size(1), 3, 3):
        return False
    H, W = x.size(2), x.size(3)
    return (x.size(1) % 64 == 0 and w.size(0) % 64 == 0 and H % 2 == 0 and W % 2 == 0 and 2 <= W <= _K13_S2_MAX_W
            and H <= 4 * _K13_S2_MAX_W)


class _Conv3x3S2Fn(torch.autograd.Function):
    """3x3 / stride 2 / pad 1 convolution: K13's stride-2 forward (the halo is rows 2r-1 .. 2r+1 of
    each output row r, still one contiguous NHWC range) with the BatchNorm statistics in its
    epilogue; both gradients on the library (convolution_backward)."""

    @staticmethod
    def forward(ctx, x, w, stats):
        y, part = torch.ops.madnn.conv3x3_fwd_s2(x, _cl(w), bool(stats))
        ctx.save_for_backward(x, w)
        ctx.mark_non_differentiable(part)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        x, w = ctx.saved_tensors
        dy = _nhwc(dy.to(x.dtype))
        dx, dw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, (2, 2), (1, 1), (1, 1), False, (0, 0), 1,
                                                        (ctx.needs_input_grad[0], ctx.needs_input_grad[1], False))
        return dx, dw, None


def conv3x3_s2(x: torch.Tensor, w: torch.Tensor, *, stats: bool = False):
    """``conv2d(x, w, stride=2, padding=1)`` of an NHWC bf16 HIP tensor, forward on K13 (see
    :func:`conv3x3_s2_supported`); ``stats`` as in :func:`conv3x3`."""
    _need_native("conv3x3_s2")
    y, part = _Conv3x3S2Fn.apply(x, w, stats)
    return (y, part) if stats else y


# ---------------------------------------------------------------------- K10
_K10 = os.environ.get("MADNN_STEM", "1") != "0"


def stem_supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Inputs the K10 stem kernels take: NHWC bf16 HIP image [N, 3, H, W] (W % 8 == 0, W <= 250),
    bf16 weight [64, 3, 7, 7]."""
    if not _K10 or x.device.type != "cuda" or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    if x.dim() != 4 or x.size(1) != 3 or tuple(w.shape) != (64, 3, 7, 7) or x.numel() == 0:
        return False
    H, W = x.size(2), x.size(3)
    return (x.is_contiguous(memory_format=torch.channels_last) and H >= 7 and W >= 8 and W % 8 == 0
            and (W - 1) // 2 + 1 <= 128 and 7 * (3 * W // 8) <= 1024)


def _stem_pack(w: torch.Tensor) -> torch.Tensor:
    """[64, 3, 7, 7] -> [64, 7 (kh), 8 (kw), 4 (c)] bf16, zero at kw = 7 and c = 3."""
    wp = w.new_zeros((64, 7, 8, 4))
    wp[:, :, :7, :3] = w.permute(0, 2, 3, 1)
    return wp


class _StemFn(torch.autograd.Function):
    """ResNet stem, 7x7 / stride 2 / pad 3, 3 -> 64 channels (K10): MFMA implicit GEMM forward
    with the BatchNorm statistics in its epilogue; MFMA weight gradient reading the im2col
    fragments straight from LDS-staged input rows.  The input gradient (never needed for an
    image batch) goes to MIOpen."""

    @staticmethod
    def forward(ctx, x, w, stats):
        y, part = torch.ops.madnn.stem_fwd(x, _stem_pack(w), bool(stats))
        ctx.save_for_backward(x, w)
        ctx.mark_non_differentiable(part)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        x, w = ctx.saved_tensors
        dy = _nhwc(dy.to(x.dtype))
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(dy, x, w, None, (2, 2), (3, 3), (1, 1), False, (0, 0), 1,
                                                     (True, False, False))[0]
        if ctx.needs_input_grad[1]:
            dw = torch.ops.madnn.stem_wgrad(dy, x).to(w.dtype)
            if not dw.is_contiguous(memory_format=torch.contiguous_format) or w.stride() != dw.stride():
                dw = torch.empty_like(w).copy_(dw)
        return dx, dw, None


def stem_conv(x: torch.Tensor, w: torch.Tensor, *, stats: bool = False):
    """``conv2d(x, w, stride=2, padding=3)`` for the ResNet stem on K10 (see
    :func:`stem_supported`).  ``stats``: also return the per-workgroup channel (sum, sum of
    squares) partials of y for :func:`batch_norm_act`."""
    _need_native("stem_conv")
    y, part = _StemFn.apply(x, w, stats)
    return (y, part) if stats else y


def hidden_supported(h: int) -> bool:
    return h % 8 == 0 and h <= 16384


__all__ = [
    "bucket_pack", "bucket_unpack", "flat_scale_cast", "sgd_step", "adam_step", "grad_norm", "layer_norm",
    "rms_norm", "batch_norm_act", "bn_supported", "cross_entropy", "attention", "attention_qkvpacked", "attention_supported",
    "max_pool2d", "max_pool_supported", "conv1x1", "conv1x1_route", "batch_norm_add_bn_relu",
    "batch_norm_dual_supported", "bn_relu_conv1x1", "bn_relu_maxpool",
    "bn_relu_maxpool_supported", "bn_relu_conv3x3", "bn_relu_conv3x3_supported",
    "bn_relu_conv1x1_epi_supported", "conv1x1_supported", "stem_conv", "stem_supported", "native_available", "load_kernels", "kernels_path", "hidden_supported", "reference",
]

if os.environ.get("MADNN_EAGER_LOAD", "0") == "1":
    load_kernels()


# --------------------------------------------------------------------------- K11
FUSED_LINEAR = os.environ.get("MADNN_FUSED_LINEAR", "1") != "0"  # models.common.linear routing (A/B switch)

def _gelu_tanh_grad(p: torch.Tensor) -> torch.Tensor:
    k0, k1 = 0.7978845608028654, 0.044715
    t = torch.tanh(k0 * (p + k1 * p * p * p))
    return 0.5 * (1 + t) + 0.5 * p * (1 - t * t) * k0 * (1 + 3 * k1 * p * p)


GELU_KIND = {"tanh": 1, "none": 2}   # F.gelu's ``approximate`` -> the kernels' GELU kind (gelu.h)


def _gelu_grad_ref(p: torch.Tensor, kind: int) -> torch.Tensor:
    if kind == 1:
        return _gelu_tanh_grad(p)
    cdf = 0.5 * (1.0 + torch.erf(p * 0.7071067811865476))
    return cdf + p * torch.exp(-0.5 * p * p) * 0.3989422804014327


def bias_grad(dy: torch.Tensor, pre: Optional[torch.Tensor] = None, bias_dtype: Optional[torch.dtype] = None,
              kind: int = 1):
    """A Linear's bias gradient: the column sum of ``dy`` over every leading dim (K11, bias.hip).

    With ``pre`` (the GELU input; ``kind`` 1 tanh / 2 erf GELU) the GELU backward is fused into the
    same pass: returns ``(db, dp)`` with ``dp = dy * gelu'(pre)`` and ``db = sum(dp)``; otherwise
    ``(db, None)``."""
    bias_dtype = bias_dtype or dy.dtype
    n = dy.shape[-1]
    if not _is_dev(dy) or n % 8:
        acc = torch.promote_types(dy.dtype, torch.float32)
        g = dy.to(acc)
        if pre is not None:
            g = g * _gelu_grad_ref(pre.to(acc), kind)
        return g.reshape(-1, n).sum(0).to(bias_dtype), (g.to(dy.dtype) if pre is not None else None)
    db, dp = _need_native("bias_grad").bias_grad(dy, pre, bias_dtype, kind)
    return db, (dp.view(dy.shape) if pre is not None else None)


GELU_KERNEL = os.environ.get("MADNN_GELU_KERNEL", "1") != "0"  # K11 GELU forward (A/B switch)


def gelu_tanh(x: torch.Tensor, kind: int = 1) -> torch.Tensor:
    """GELU forward (``kind`` 1: tanh approximation, 2: exact erf): the K11-family streaming kernel
    on HIP tensors (16-byte accesses, v_exp-based), ``F.gelu`` elsewhere.  No autograd: the caller
    (the fused Linear / MLP) saves the pre-activation and runs the GELU backward in K11 / K12P."""
    if GELU_KERNEL and _is_dev(x) and x.numel() % 8 == 0 and x.dtype in (torch.bfloat16, torch.float32):
        return _need_native("gelu_tanh").gelu_fwd(x, kind)
    return F.gelu(x, approximate="tanh" if kind == 1 else "none")


def grad_sink(weight: torch.Tensor) -> Optional[torch.Tensor]:
    """Where ``weight``'s gradient should be WRITTEN: a fresh view of its slot in the data-parallel
    reducer's flat gradient bucket when (a) the parameter lives in a FlatParamSpace with sinks
    enabled, (b) its bucket reduces in the parameter's dtype and (c) no gradient was accumulated
    yet this step (``weight.grad is None``).  A layer that computes its weight gradient with a
    GEMM writes it there (``torch.mm(..., out=sink)``) and returns the view; autograd adopts it
    as ``p.grad`` without a copy and the reducer skips the K4 pack for it."""
    space = getattr(weight, "_madnn_space", None)
    if space is None or weight.grad is not None:
        return None
    return space.grad_slot(weight)


WGRAD = os.environ.get("MADNN_WGRAD", "auto")  # weight-gradient GEMM: auto (timed per shape) | lt | k12
_WGRAD_CHOICE: dict = {}
_GELU_FWD_CHOICE: dict = {}
_DGELU_CHOICE: dict = {}
_DGRAD_CHOICE: dict = {}
_TUNE = {"timed": 0, "table": None}   # run-time timings taken; the shipped table that was loaded
_TUNE_MS: dict = {}   # (table, key) -> {implementation: ms for 3 calls} of every run-time timing (the A/B record)

# Per-shape implementation choices measured on MI355X and shipped in-tree, so a job starts
# without timing anything (a first-use timing runs BOTH implementations, and a library kernel's
# first use can cost seconds of MIOpen problem search) and every replica of a multi-GPU job
# runs the same kernels.  ``scripts/record_tuning.py`` regenerates it on a GPU box.
TUNE_TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning",
                          "choices_gfx950.json")


def load_tuning_table(path: Optional[str] = None) -> int:
    """Adopt the shipped per-shape choices (``MADNN_TUNE_TABLE=0`` disables; ``MADNN_TUNE_TABLE_PATH``
    overrides the file).  Returns the number of entries loaded."""
    import ast
    import json

    if os.environ.get("MADNN_TUNE_TABLE", "1") == "0":
        return 0
    path = path or os.environ.get("MADNN_TUNE_TABLE_PATH") or TUNE_TABLE
    try:
        with open(path) as f:
            data = json.load(f)
    except (OSError, ValueError):
        return 0
    n = 0
    for name, dst in (("wgrad", _WGRAD_CHOICE), ("gelu_fwd", _GELU_FWD_CHOICE), ("dgelu", _DGELU_CHOICE),
                      ("dgrad", _DGRAD_CHOICE)):
        for k, v in data.get(name, {}).items():
            dst.setdefault(ast.literal_eval(k), v)
            n += 1
    _TUNE["table"] = path
    return n


def export_choices(path: str) -> None:
    """Write every per-shape choice this process holds (shipped + timed) in the table format."""
    import json

    data = {"arch": "gfx950", "wgrad": {repr(k): v for k, v in sorted(_WGRAD_CHOICE.items(), key=repr)},
            "gelu_fwd": {repr(k): v for k, v in sorted(_GELU_FWD_CHOICE.items(), key=repr)},
            "dgelu": {repr(k): v for k, v in sorted(_DGELU_CHOICE.items(), key=repr)},
            "dgrad": {repr(k): v for k, v in sorted(_DGRAD_CHOICE.items(), key=repr)}}
    with open(path, "w") as f:
        json.dump(data, f, indent=1)
        f.write("\n")


def sync_choices(group=None, src: int = 0) -> None:
    """Every rank of ``group`` adopts global rank ``src``'s per-shape choices, so replicas that
    timed a shape missing from the table independently still run identical kernels from here on."""
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) <= 1:
        return
    obj = [(dict(_WGRAD_CHOICE), dict(_GELU_FWD_CHOICE), dict(_DGELU_CHOICE), dict(_DGRAD_CHOICE))]
    dist.broadcast_object_list(obj, src=src, group=group)
    _WGRAD_CHOICE.update(obj[0][0])
    _GELU_FWD_CHOICE.update(obj[0][1])
    _DGELU_CHOICE.update(obj[0][2])
    _DGRAD_CHOICE.update(obj[0][3])


def tuning_timings() -> int:
    """How many per-shape timings this process ran (0 when the table covered every shape)."""
    return _TUNE["timed"]


def tuning_measurements() -> list:
    """Every per-shape timing this process ran: [{"table", "key", "ms": {impl: ms}, "chosen"}]."""
    out = []
    for (tab, key), ms in _TUNE_MS.items():
        chosen = {"wgrad": _WGRAD_CHOICE, "gelu_fwd": _GELU_FWD_CHOICE, "dgelu": _DGELU_CHOICE,
                  "dgrad": _DGRAD_CHOICE}[tab].get(key)
        out.append({"table": tab, "key": repr(key), "ms": {k: round(v, 4) for k, v in ms.items()}, "chosen": chosen})
    return out


def _wgrad_k12_ok(g2, x2, out) -> bool:
    return (_is_dev(g2) and g2.dtype == x2.dtype == out.dtype == torch.bfloat16 and g2.shape[0] % 64 == 0
            and g2.shape[1] % 8 == 0 and x2.shape[1] % 8 == 0 and g2.is_contiguous() and x2.is_contiguous()
            and out.is_contiguous() and load_kernels())


def _time_wgrad(fn, iters: int = 3) -> float:
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e)


def wgrad_into(g2: torch.Tensor, x2: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """``out[N, K] = g2[M, N]^T @ x2[M, K]``: a Linear's weight gradient, reduced over the M tokens.

    Two implementations: hipBLASLt (``torch.mm``) and K12 with the tokens split over several
    workgroups per output tile (``linear_wgrad``).  A weight gradient has few output tiles and a
    very long reduction (GPT-2 medium: 16-64 tiles of 256^2 over 65536 tokens), which leaves most
    of the 256 CUs idle unless the reduction is split; hipBLASLt's choice does not always split
    (``profiles/r3_wgrad_ab.json``: 1.9x on the attention projection, 1.15x on c_fc, 0.95x on
    c_proj).  ``MADNN_WGRAD=auto`` times both once per (M, N, K) on first use (like cuDNN's
    benchmark mode; never under graph capture) and keeps the faster."""
    lib = lambda: torch.mm(g2.t(), x2, out=out)  # noqa: E731
    if WGRAD == "lt" or not _wgrad_k12_ok(g2, x2, out):
        return lib()
    return tuned_wgrad(("linear",) + tuple(g2.shape) + (x2.shape[1],), lib,
                       lambda: torch.ops.madnn.linear_wgrad(g2, x2, out, False, 0),
                       k12w=lambda: torch.ops.madnn.linear_wgrad4(g2, x2, out, False, 0),
                       k12wh=(lambda: torch.ops.madnn.linear_wgrad4h(g2, x2, out, False, 0))
                       if g2.shape[0] % 128 == 0 else None)


def tuned_wgrad(key, lib, k12, k9=None, k12w=None, k12wh=None):
    """Run the weight-gradient implementation that was faster for ``key``: ``lib`` (the library
    kernel: hipBLASLt / MIOpen), ``k12`` (K12 split-K over the rows), ``k12w`` (K12W: the same
    split-K GEMM at one wave per SIMD, 128 x 128 per wave, on ``v_mfma_f32_32x32x16_bf16``), ``k12wh``
    (K12W16: its ``v_mfma_f32_16x16x32_bf16`` form, rows a multiple of 128) or, for NHWC 1x1
    convolutions, ``k9`` (K9's split-M kernel, slabs reduced and cast in one pass) -- from the shipped
    table (:func:`load_tuning_table`), else timed once on first use (outside graph capture).
    ``MADNN_WGRAD=lt`` / ``k12`` / ``k12w`` / ``k12wh`` pin one."""
    if WGRAD == "lt":
        return lib()
    if WGRAD == "k12":
        return k12()
    if WGRAD == "k12w" and k12w is not None:
        return k12w()
    if WGRAD == "k12wh" and k12wh is not None:
        return k12wh()
    cands = {"lib": lib, "k12": k12}
    if k12w is not None:
        cands["k12w"] = k12w
    if k12wh is not None:
        cands["k12wh"] = k12wh
    if k9 is not None:
        cands["k9"] = k9
    choice = _WGRAD_CHOICE.get(key)
    if choice not in cands:
        if torch.cuda.is_current_stream_capturing():
            return lib()
        _TUNE["timed"] += 1
        times = {k: _time_wgrad(f) for k, f in cands.items()}
        _TUNE_MS[("wgrad", key)] = times
        choice = _WGRAD_CHOICE[key] = min(times, key=times.get)
    return cands[choice]()


def _k9_wgrad(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """K9's weight gradient in ``w``'s dtype (the split reduction writes it: no cast pass)."""
    return torch.ops.madnn.conv1x1_wgrad(dy, x, w.dtype == torch.bfloat16).to(w.dtype).view(w.shape)


def _conv1x1_wgrad_lib(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """The 1x1 convolution's weight gradient on the library path: MIOpen's wrw for NHWC 4-D
    tensors, hipBLASLt for 2-D rows -- or K12 split-K over the pixels when that was faster for
    the shape (:func:`tuned_wgrad`)."""
    if x.dim() == 4:
        lib = lambda: torch.ops.aten.convolution_backward(  # noqa: E731
            dy, x, w.view(w.size(0), -1, 1, 1), None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1,
            (False, True, False))[1].view(w.shape)
    else:
        lib = lambda: torch.mm(dy.t(), x).view(w.shape)  # noqa: E731
    dr, xr = _rows(dy), _rows(x)
    probe = torch.empty(0, dtype=w.dtype, device=w.device)
    if not _wgrad_k12_ok(dr, xr, probe) or w.dtype != torch.bfloat16:
        return lib()
    k9 = (lambda: _k9_wgrad(dy, x, w)) if x.dim() == 4 and conv1x1_supported(x, w.view(w.size(0), -1)) else None
    return tuned_wgrad(("conv1x1", dr.shape[0], dr.shape[1], xr.shape[1]), lib,
                       lambda: torch.ops.madnn.linear_wgrad(dr, xr, None, False, 0).view(w.shape), k9,
                       k12w=lambda: torch.ops.madnn.linear_wgrad4(dr, xr, None, False, 0).view(w.shape),
                       k12wh=(lambda: torch.ops.madnn.linear_wgrad4h(dr, xr, None, False, 0).view(w.shape))
                       if dr.shape[0] % 128 == 0 else None)


LT_EPILOGUE = os.environ.get("MADNN_LT_EPILOGUE", "1") != "0"  # hipBLASLt GELU/residual epilogues (A/B switch)
_LT_FAILED = {}   # (gelu, residual) -> the error that disabled that epilogue kind
_LT_KIND = {"gelu": os.environ.get("MADNN_LT_GELU", "1") != "0", "res": os.environ.get("MADNN_LT_RES", "1") != "0"}


def _lt_ok(x: torch.Tensor, weight: torch.Tensor, gelu: bool = False, residual: bool = False) -> bool:
    if gelu and not _LT_KIND["gelu"] or residual and not _LT_KIND["res"]:
        return False
    return (LT_EPILOGUE and (bool(gelu), bool(residual)) not in _LT_FAILED and x.dtype == torch.bfloat16
            and weight.dtype == torch.bfloat16 and x.is_cuda and weight.is_contiguous())


def _lt_linear(x2, weight, bias, residual, gelu):
    """(y, pre) from one hipBLASLt call with the bias / GELU(+aux) / residual epilogue, or None
    if hipBLASLt refuses it (then that epilogue kind uses the unfused path for good)."""
    try:
        y, pre = _need_native("lt_linear").lt_linear(x2, weight, bias, residual, bool(gelu), bool(gelu))
        return y, (pre if gelu else None)
    except RuntimeError as e:  # noqa: PERF203 - once per kind
        _LT_FAILED[(bool(gelu), residual is not None)] = e
        import sys

        print(f"[madnn] hipBLASLt epilogue (gelu={gelu}, residual={residual is not None}) disabled: {e}",
              file=sys.stderr)
        return None


GELU_FWD = os.environ.get("MADNN_GELU_FWD", "auto")  # GELU Linear forward: auto (timed per shape) | lt | k12


def _k12_fwd_ok(x2: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> bool:
    return (_is_dev(x2) and x2.dtype == weight.dtype == torch.bfloat16 and x2.is_contiguous()
            and weight.is_contiguous() and x2.shape[1] % 64 == 0 and weight.shape[0] % 8 == 0
            and x2.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0
            and (bias is None or (bias.is_contiguous() and bias.dtype in (torch.float32, torch.bfloat16)))
            and load_kernels())


def _k12p_ok(rows: torch.Tensor, weight: torch.Tensor, out_features: int, tokens: int, red: int,
             has_bias: bool) -> bool:
    """K12P (the persistent GEMM with fused epilogues, gemmp.hip) takes the shape: 256-multiples
    of tokens and output features (no edge tiles), a 64-multiple reduction, contiguous 16-B aligned
    bf16 operands."""
    return (_is_dev(rows) and rows.dtype == weight.dtype == torch.bfloat16 and rows.is_contiguous()
            and weight.is_contiguous() and rows.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0
            and load_kernels() and bool(torch.ops.madnn.gemmp_supported(out_features, tokens, red, has_bias)))


def _timed_choice(table: dict, key, cands: dict, default: str) -> str:
    """The implementation in ``cands`` that was faster for ``key`` (shipped table, else timed
    once on first use outside graph capture, like :func:`tuned_wgrad`)."""
    choice = table.get(key)
    if choice in cands:
        return choice
    if torch.cuda.is_current_stream_capturing():
        return default
    _TUNE["timed"] += 1
    times = {k: _time_wgrad(f) for k, f in cands.items()}
    name = {id(_GELU_FWD_CHOICE): "gelu_fwd", id(_DGELU_CHOICE): "dgelu", id(_DGRAD_CHOICE): "dgrad"}[id(table)]
    _TUNE_MS[(name, key)] = times
    choice = table[key] = min(times, key=times.get)
    return choice


def _gelu_linear_fwd(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], kind: int = 1):
    """``(gelu(pre), pre)`` with ``pre = x W^T + b`` (``kind`` 1 tanh / 2 erf GELU), from whichever
    implementation was faster for the shape (timed once on first use, like :func:`tuned_wgrad`):

    * ``lt``: hipBLASLt GEMM (bias epilogue), then the K11 streaming GELU pass (hipBLASLt has no
      GELU+AUX algorithm at GPT-2's 65536-row shapes on gfx950);
    * ``k12p``: K12P, the persistent GEMM whose epilogue adds the bias, stores the pre-activation
      (the backward's AUX) and the GELU output from the accumulators while the next tile's
      operands stream in (on shapes without edge tiles);
    * ``k12``: the one-tile-per-workgroup K12 with the same epilogue staged through LDS (other
      shapes).

    ``MADNN_GELU_FWD=lt`` / ``k12`` / ``k12p`` pin one."""
    x2 = x.reshape(-1, x.shape[-1])
    out_shape = (*x.shape[:-1], weight.shape[0])

    def lt():
        pre = F.linear(x2, weight, bias if bias is None or bias.dtype == x2.dtype else bias.to(x2.dtype))
        return gelu_tanh(pre, kind), pre

    def k12():
        return torch.ops.madnn.linear_fwd(x2, weight, bias, None, kind, True)

    def k12p():
        return torch.ops.madnn.linear_fwd_p(x2, weight, bias, kind)

    tag = () if kind == 1 else ("erf",)

    ok12 = _k12_fwd_ok(x2, weight, bias)
    okp = ok12 and _k12p_ok(x2, weight, weight.shape[0], x2.shape[0], x2.shape[1], bias is not None)
    choice = GELU_FWD
    if choice == "k12p" and not okp or choice == "k12" and not ok12:
        choice = "lt"
    if choice not in ("lt", "k12", "k12p"):
        choice = "lt"
        if okp:
            key = ("p", tuple(x2.shape), tuple(weight.shape), bias is not None) + tag
            choice = _timed_choice(_GELU_FWD_CHOICE, key, {"lt": lt, "k12p": k12p}, "lt")
        elif ok12:
            key = (tuple(x2.shape), tuple(weight.shape), bias is not None) + tag
            choice = _timed_choice(_GELU_FWD_CHOICE, key, {"lt": lt, "k12": k12}, "lt")
    y, pre = {"lt": lt, "k12": k12, "k12p": k12p}[choice]()
    return y.view(out_shape), pre.view(out_shape)


DGELU = os.environ.get("MADNN_DGELU", "auto")  # c_proj dgrad + GELU backward: auto | lt | k12p


def dgrad_dgelu(g2: torch.Tensor, w2: torch.Tensor, pre2: torch.Tensor, bias_dtype: torch.dtype, kind: int = 1):
    """``(dh, db)``: the data gradient of the Linear after a GELU (``kind`` 1 tanh / 2 erf;
    ``da = g2 @ w2``) pushed
    through that GELU (``dh = da * gelu'(pre)``) plus the GELU Linear's bias gradient
    (``db = sum(dh)``), from whichever was faster for the shape:

    * ``lt``: hipBLASLt GEMM, then the K11 dGELU + column-sum pass (reads ``da`` and ``pre``,
      writes ``dh``);
    * ``k12p``: K12P with the dGELU epilogue -- ``da`` never reaches HBM, the column sums come from
      the accumulators (per-wave partial rows + one finalize).

    ``MADNN_DGELU=lt`` / ``k12p`` pin one."""
    def lt():
        db, dh = bias_grad(g2 @ w2, pre2, bias_dtype, kind)
        return dh, db

    def k12p():
        return tuple(torch.ops.madnn.linear_dgrad_p(g2, w2, pre2, bias_dtype, kind))

    ok = (bias_dtype in (torch.float32, torch.bfloat16) and _is_dev(pre2) and pre2.dtype == g2.dtype
          and pre2.is_contiguous() and pre2.data_ptr() % 16 == 0
          and _k12p_ok(g2, w2, w2.shape[1], g2.shape[0], g2.shape[1], False))
    choice = DGELU if DGELU in ("lt", "k12p") else "auto"
    if choice == "k12p" and not ok:
        choice = "lt"
    if choice == "auto":
        choice = "lt"
        if ok:
            key = (tuple(g2.shape), tuple(w2.shape), str(bias_dtype)) + (() if kind == 1 else ("erf",))
            choice = _timed_choice(_DGELU_CHOICE, key, {"lt": lt, "k12p": k12p}, "lt")
    return lt() if choice == "lt" else k12p()


DGRAD = os.environ.get("MADNN_DGRAD", "auto")  # plain Linear data gradient: auto | lt | ltk | k12p


def dgrad(g2: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """``g2 @ weight``: a Linear's data gradient, from whichever was faster for the shape (shipped
    table, else timed once on first use like :func:`tuned_wgrad`):

    * ``lt``: PyTorch's matmul (hipBLASLt through PyTorch's own plan);
    * ``ltk``: madnn's hipBLASLt plan for the same product (``lt_linear(..., w_kn=True)``: the weight
      taken as [K, N] without a transposed copy) -- the same library, but its plan picks a different
      kernel on some shapes: the GPT-2 qkv data gradient runs 713 us there against 838 us through
      PyTorch (``profiles/r6_lt_algo_sweep.jsonl``);
    * ``k12p``: the persistent K12P GEMM, plain epilogue (hipBLASLt's choice at 32k-token microbatches
      ran the GPT-2 data gradients 35 % slower per FLOP than at 131k tokens,
      ``profiles/r6_gpt2m_mb32_steady_steps.md``).

    ``MADNN_DGRAD=lt`` / ``ltk`` / ``k12p`` pin one."""
    def lt():
        return g2 @ weight

    if DGRAD == "lt" or not (g2.is_contiguous() and weight.is_contiguous() and _is_dev(g2)
                             and g2.dtype == weight.dtype == torch.bfloat16):
        return lt()

    def ltk():
        return _need_native("lt_linear").lt_linear(g2, weight, None, None, False, False, True)[0]

    cands = {"lt": lt, "ltk": ltk}
    if _k12p_ok(g2, weight, weight.shape[1], g2.shape[0], g2.shape[1], False):
        def k12p():
            return torch.ops.madnn.linear_dgrad_p(g2, weight, None, g2.dtype, 1)[0]
        cands["k12p"] = k12p
    if DGRAD in cands:
        return cands[DGRAD]()
    key = (tuple(g2.shape), tuple(weight.shape))
    return cands[_timed_choice(_DGRAD_CHOICE, key, cands, "lt")]()


class _LinearFn(torch.autograd.Function):
    """y = act(x W^T + b) (+ residual) with act in {identity, tanh-GELU}.

    Forward: one hipBLASLt GEMM whose epilogue adds the bias, applies the GELU (keeping the
    pre-activation as its AUX output for the backward) and adds the residual stream -- no
    standalone elementwise passes.  Backward: the bias gradient (and the GELU backward) come from
    one K11 pass, the data-gradient GEMM stays on hipBLASLt, and the weight-gradient GEMM
    (:func:`wgrad_into`: hipBLASLt or K12 split-K, whichever is faster for the shape) writes straight
    into the reducer's bucket when the weight has a :func:`grad_sink`; the residual's gradient is
    the output gradient itself (no copy)."""

    @staticmethod
    def forward(ctx, x, weight, bias, gelu, residual):
        ctx.gelu = gelu
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.param = weight  # the Parameter itself (for its grad sink); not modified before backward
        ctx.has_res = residual is not None
        out = None
        if (gelu or residual is not None) and _lt_ok(x, weight, gelu, residual is not None):
            x2 = x.reshape(-1, x.shape[-1])
            if not x2.is_contiguous():
                x2 = x2.contiguous()
            r2 = residual.reshape(-1, weight.shape[0]).contiguous() if residual is not None else None
            out = _lt_linear(x2, weight, bias if bias is None or bias.is_contiguous() else bias.contiguous(), r2, gelu)
        if out is not None:
            y, pre = out
            y = y.view(*x.shape[:-1], weight.shape[0])
            if gelu:
                ctx.save_for_backward(x, weight, pre.view_as(y))
            else:
                ctx.save_for_backward(x, weight)
            return y
        if gelu:
            y, pre = _gelu_linear_fwd(x, weight, bias)
            ctx.save_for_backward(x, weight, pre)
            return y + residual if residual is not None else y
        pre = F.linear(x, weight, bias)
        if gelu:
            ctx.save_for_backward(x, weight, pre)
            y = gelu_tanh(pre)
        else:
            ctx.save_for_backward(x, weight)
            y = pre
        return y + residual if residual is not None else y

    @staticmethod
    def backward(ctx, g):
        if ctx.gelu:
            x, weight, pre = ctx.saved_tensors
        else:
            (x, weight), pre = ctx.saved_tensors, None
        db = None
        g_out = g   # the residual's gradient: the upstream gradient itself, not the GELU-scaled one
        if ctx.gelu:
            db, g = bias_grad(g, pre, ctx.bias_dtype or g.dtype)
            if ctx.bias_dtype is None:
                db = None
        elif ctx.bias_dtype is not None and ctx.needs_input_grad[2]:
            # from the consumer's backward (_NormFn, _AttnPackedFn); a reshaped view keeps it on its base
            cs = _attached(g, "_madnn_colsum")
            if cs is not None and cs.numel() == g.shape[-1]:
                db = cs.to(ctx.bias_dtype)
            else:
                db, _ = bias_grad(g, None, ctx.bias_dtype)
        g2 = g.reshape(-1, g.shape[-1])
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = dgrad(g2, weight).view(*x.shape[:-1], weight.shape[1])
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, x.shape[-1])
            sink = grad_sink(ctx.param)
            if sink is not None and sink.dtype == g2.dtype == x2.dtype and sink.is_contiguous():
                dw = wgrad_into(g2, x2, sink)
            elif weight.dtype == g2.dtype == x2.dtype and _is_dev(g2):
                dw = wgrad_into(g2, x2, torch.empty(weight.shape, dtype=weight.dtype, device=weight.device))
            else:
                dw = (g2.t() @ x2).to(weight.dtype)
        ctx.param = None
        return dx, dw, db, None, (g_out if ctx.has_res else None)


def _linear_residual_fwd(a: torch.Tensor, weight, bias, residual):
    """``a W^T + b (+ residual)``: one hipBLASLt call with the bias / residual epilogue when it
    takes it, else ``F.linear`` + add."""
    if _lt_ok(a, weight, False, residual is not None):
        a2 = a.reshape(-1, a.shape[-1])
        if not a2.is_contiguous():
            a2 = a2.contiguous()
        r2 = residual.reshape(-1, weight.shape[0]).contiguous() if residual is not None else None
        out = _lt_linear(a2, weight, bias if bias is None or bias.is_contiguous() else bias.contiguous(), r2, False)
        if out is not None:
            return out[0].view(*a.shape[:-1], weight.shape[0])
    # an fp32 bias (kept in fp32 by the data-parallel space) joins a bf16 GEMM in the GEMM's dtype
    y = F.linear(a, weight, bias if bias is None or bias.dtype == a.dtype else bias.to(a.dtype))
    return y + residual if residual is not None else y


_LT_KN_FAILED = []  # the [K, N]-weight residual GEMM was refused once: addmm from then on


def _dgrad_plus(g2: torch.Tensor, weight: torch.Tensor, res2: torch.Tensor) -> torch.Tensor:
    """``g2 @ weight + res2`` (a data gradient plus a residual path's gradient) as ONE hipBLASLt GEMM
    reading the [out, in] weight as it is stored (op N) and res2 as its C operand -- not ``addmm``,
    which first copies res2 (rows x features) into its output."""
    if not _LT_KN_FAILED and _lt_ok(g2, weight, False, True) and g2.is_contiguous():
        try:
            y, _ = _need_native("lt_linear").lt_linear(g2, weight, None, res2.contiguous().to(g2.dtype), False, False,
                                                       True)
            return y
        except RuntimeError as e:  # noqa: PERF203 - once
            _LT_KN_FAILED.append(e)
    return torch.addmm(res2.to(g2.dtype), g2, weight)


class _LinearTeeFn(torch.autograd.Function):
    """``(x W^T + b, x)``: a Linear whose input also feeds a residual path (BERT's post-LN attention
    sublayer, LN(x + attn(x))).  Both uses of x are this node, so the residual's gradient (the second
    output's) joins the data-gradient GEMM as its C operand (beta = 1) instead of a separate
    accumulation pass over x's two gradients.  Bias gradient and weight gradient as _LinearFn."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.param = weight
        ctx.save_for_backward(x, weight)
        return _linear_residual_fwd(x, weight, bias, None), x.view_as(x)

    @staticmethod
    def backward(ctx, g, gx):
        x, weight = ctx.saved_tensors
        db = None
        if ctx.bias_dtype is not None and ctx.needs_input_grad[2]:
            cs = _attached(g, "_madnn_colsum")  # the attention backward's dQKV column sums
            if cs is not None and cs.numel() == g.shape[-1]:
                db = cs.to(ctx.bias_dtype)
            else:
                db, _ = bias_grad(g, None, ctx.bias_dtype)
        g2 = g.reshape(-1, g.shape[-1])
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if gx is None:
                dx = g2 @ weight
            else:
                dx = _dgrad_plus(g2, weight, gx.reshape(-1, weight.shape[1]))
            dx = dx.view(*x.shape[:-1], weight.shape[1])
        if ctx.needs_input_grad[1]:
            dw = _weight_grad(g2, x.reshape(-1, x.shape[-1]), ctx.param)
        ctx.param = None
        return dx, dw, db


def linear_tee(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None):
    """``(F.linear(x, weight, bias), x')`` where ``x'`` is ``x`` for a residual path whose gradient
    is summed inside this Linear's data-gradient GEMM (:class:`_LinearTeeFn`); eager on CPU."""
    if not torch.is_grad_enabled() or not _is_dev(x) or weight.shape[0] % 8:
        return F.linear(x, weight, bias if bias is None or bias.dtype == x.dtype else bias.to(x.dtype)), x
    return _LinearTeeFn.apply(x, weight, bias)


def _weight_grad(g2: torch.Tensor, x2: torch.Tensor, param: torch.Tensor) -> torch.Tensor:
    """A Linear's weight gradient, written into the reducer's bucket slot when it has one."""
    sink = grad_sink(param)
    if sink is not None and sink.dtype == g2.dtype == x2.dtype and sink.is_contiguous():
        return wgrad_into(g2, x2, sink)
    if param.dtype == g2.dtype == x2.dtype and _is_dev(g2):
        return wgrad_into(g2, x2, torch.empty(param.shape, dtype=param.dtype, device=param.device))
    return (g2.t() @ x2).to(param.dtype)


class _GeluMLPFn(torch.autograd.Function):
    """``c_proj(gelu_tanh(c_fc(x))) (+ residual)`` as ONE autograd node, so that the GELU's
    activation has no other consumer and its backward can live inside c_proj's data-gradient GEMM.

    Forward: c_fc + bias + GELU in one GEMM epilogue (:func:`_gelu_linear_fwd`: K12P stores the
    pre-activation and the activation from the accumulators), c_proj + bias + residual in
    hipBLASLt's epilogue.  Backward: c_proj's bias gradient (the consumer's column sum when
    attached), c_proj's weight gradient, then :func:`dgrad_dgelu` -- c_proj's data gradient with
    c_fc's GELU backward and c_fc's bias gradient in its epilogue (no ``da`` in HBM, no K11
    pass) -- and c_fc's weight and data gradients.  Weight gradients go straight into the
    data-parallel buckets (:func:`grad_sink`).  Reference: the MP layer pair's activation
    (nodemodule.lua:133-159)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, residual, kind=1):
        a, pre = _gelu_linear_fwd(x, w1, b1, kind)
        ctx.kind = kind
        y = _linear_residual_fwd(a, w2, b2, residual)
        ctx.save_for_backward(x, w1, pre, a, w2)
        ctx.b1_dtype = b1.dtype if b1 is not None else None
        ctx.b2_dtype = b2.dtype if b2 is not None else None
        ctx.bias_dtype = ctx.b2_dtype   # the output's bias: consumers attach its column sum (_linear_bias_dtype)
        ctx.params = (w1, w2)
        ctx.has_res = residual is not None
        # the residual IS the input (a post-LN block: y + MLP(y)): its gradient is added inside the
        # input's data-gradient GEMM (beta = 1) instead of by autograd's accumulation pass
        ctx.res_is_x = residual is x
        return y

    @staticmethod
    def backward(ctx, g):
        x, w1, pre, a, w2 = ctx.saved_tensors
        p1, p2 = ctx.params
        ctx.params = None
        need = ctx.needs_input_grad
        db2 = None
        if ctx.b2_dtype is not None and need[4]:
            cs = _attached(g, "_madnn_colsum")
            if cs is not None and cs.numel() == g.shape[-1]:
                db2 = cs.to(ctx.b2_dtype)
            else:
                db2, _ = bias_grad(g, None, ctx.b2_dtype)
        g2 = g.reshape(-1, g.shape[-1])
        if not g2.is_contiguous():
            g2 = g2.contiguous()
        a2 = a.reshape(-1, a.shape[-1])
        dw2 = _weight_grad(g2, a2, p2) if need[3] else None
        dh, db1 = dgrad_dgelu(g2, w2, pre.reshape(-1, pre.shape[-1]), ctx.b1_dtype or g2.dtype, ctx.kind)
        if ctx.b1_dtype is None or not need[2]:
            db1 = None
        x2 = x.reshape(-1, x.shape[-1])
        dw1 = _weight_grad(dh, x2, p1) if need[1] else None
        if ctx.res_is_x and need[0]:
            dx = _dgrad_plus(dh, w1, g2).view(*x.shape[:-1], w1.shape[1])
            return dx, dw1, db1, dw2, db2, None, None
        dx = (dh @ w1).view(*x.shape[:-1], w1.shape[1]) if need[0] else None
        return dx, dw1, db1, dw2, db2, (g if ctx.has_res else None), None


def gelu_mlp(x: torch.Tensor, w1: torch.Tensor, b1: Optional[torch.Tensor], w2: torch.Tensor,
             b2: Optional[torch.Tensor], residual: Optional[torch.Tensor] = None,
             approximate: str = "tanh") -> torch.Tensor:
    """``linear(gelu(linear(x, w1, b1)), w2, b2) (+ residual)``: the transformer MLP as one fused
    autograd node on HIP tensors (:class:`_GeluMLPFn`), eager ops elsewhere.  ``approximate`` as
    in ``F.gelu``: "tanh" (GPT-2) or "none" (the exact erf GELU, BERT)."""
    if residual is not None and residual.shape[:-1] != x.shape[:-1]:
        raise ValueError("gelu_mlp: residual must have the output's shape")
    if approximate not in GELU_KIND:
        raise ValueError(f"gelu_mlp: approximate must be 'tanh' or 'none', not {approximate!r}")
    if not _is_dev(x) or not torch.is_grad_enabled() or w1.shape[0] % 8 or w2.shape[0] % 8:
        h = F.gelu(F.linear(x, w1, b1), approximate=approximate)
        y = F.linear(h, w2, b2)
        return y + residual if residual is not None else y
    return _GeluMLPFn.apply(x, w1, b1, w2, b2, residual, GELU_KIND[approximate])


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None, gelu: bool = False,
           force_fn: bool = False, residual: Optional[torch.Tensor] = None):
    """``act(F.linear(x, weight, bias)) + residual`` with act in {identity, tanh-GELU}: one
    epilogue-fused hipBLASLt GEMM forward; backward fuses the bias gradient (K11) and writes the
    weight gradient into the reducer bucket (:func:`grad_sink`).  Eager ops on CPU tensors
    (``force_fn`` runs the autograd Function anyway: tests of the sink path)."""
    if residual is not None and residual.shape[:-1] != x.shape[:-1]:
        raise ValueError("linear: residual must have the output's shape")
    if not torch.is_grad_enabled() or (not force_fn and (not _is_dev(x) or weight.shape[0] % 8)):
        if not torch.is_grad_enabled() and _is_dev(x) and (gelu or residual is not None) \
                and _lt_ok(x, weight, gelu, residual is not None) \
                and weight.shape[0] % 8 == 0:
            x2 = x.reshape(-1, x.shape[-1]).contiguous()
            r2 = residual.reshape(-1, weight.shape[0]).contiguous() if residual is not None else None
            out = _lt_linear(x2, weight, bias, r2, gelu)
            if out is not None:
                return out[0].view(*x.shape[:-1], weight.shape[0])
        y = F.linear(x, weight, bias)
        y = F.gelu(y, approximate="tanh") if gelu else y
        return y + residual if residual is not None else y
    return _LinearFn.apply(x, weight, bias, gelu, residual)


load_tuning_table()
