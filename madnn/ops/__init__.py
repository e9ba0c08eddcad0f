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

from . import reference

HERE = Path(__file__).resolve().parent
_KERNELS = HERE / "_madnn_kernels.so"
_lock = threading.Lock()
_loaded = {"kernels": False, "error": None}


def kernels_path() -> Path:
    return _KERNELS


def load_kernels(build_if_missing: bool = True) -> bool:
    """Load the HIP kernel library (building it in-tree if absent and hipcc exists)."""
    with _lock:
        if _loaded["kernels"]:
            return True
        try:
            if not _KERNELS.exists() and build_if_missing:
                from .build import build

                build()
            torch.ops.load_library(str(_KERNELS))
            _loaded["kernels"] = True
            _loaded["error"] = None
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
    @staticmethod
    def forward(ctx, x, res, w, b, eps, rms):
        shape = x.shape
        xc = x.contiguous()
        rc = res.contiguous() if res is not None else None
        y, s, mean, rstd = _need_native("norm_fwd").norm_fwd(xc, rc, w, b, float(eps), bool(rms))
        saved_x = s if res is not None else xc
        ctx.save_for_backward(saved_x, w, mean, rstd)
        ctx.rms = rms
        ctx.has_bias = b is not None
        ctx.has_res = res is not None
        ctx.shape = shape
        if res is not None:
            return y.view(shape), s.view(shape)
        return y.view(shape), None

    @staticmethod
    def backward(ctx, dy, ds):
        x, w, mean, rstd = ctx.saved_tensors
        dres = ds.contiguous() if (ctx.has_res and ds is not None) else None
        dx, dw, db = torch.ops.madnn.norm_bwd(dy.contiguous(), x, w, mean, rstd, dres, ctx.rms, ctx.has_bias)
        dx = dx.view(ctx.shape)
        return dx, (dx if ctx.has_res else None), dw, (db if ctx.has_bias else None), None, None


def _norm(x, weight, bias, eps, rms, residual):
    if _is_dev(x):
        if weight is None:
            raise ValueError("madnn norm kernels need an affine weight")
        y, s = _NormFn.apply(x, residual, weight, bias, eps, rms)
        return (y, s) if residual is not None else y
    return reference.norm(x, weight, bias, eps, rms, residual)


def layer_norm(x, weight, bias=None, eps: float = 1e-5, residual: Optional[torch.Tensor] = None):
    """LayerNorm over the last dim.  With ``residual``: returns (LN(x + residual), x + residual)."""
    return _norm(x, weight, bias, eps, False, residual)


def rms_norm(x, weight, eps: float = 1e-6, residual: Optional[torch.Tensor] = None):
    """RMSNorm over the last dim.  With ``residual``: returns (RMS(x + residual), x + residual)."""
    return _norm(x, weight, None, eps, True, residual)


def hidden_supported(h: int) -> bool:
    return h % 8 == 0 and h <= 16384


__all__ = [
    "bucket_pack", "bucket_unpack", "flat_scale_cast", "sgd_step", "adam_step", "grad_norm", "layer_norm",
    "rms_norm", "native_available", "load_kernels", "kernels_path", "hidden_supported", "reference",
]

if os.environ.get("MADNN_EAGER_LOAD", "0") == "1":
    load_kernels()
