"""Eager PyTorch references for every madnn kernel.

Used (a) on CPU tensors, where the gloo tier of the test suite runs, and (b)
as the fp32 numerics oracle in the GPU kernel tests.  Semantics are the
kernels' exactly (same argument order, same optional fused pieces).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch


def is_dense(t: torch.Tensor) -> bool:
    """True if ``t`` covers one gap-free, non-overlapping block of memory (any stride order)."""
    expected = 1
    for d in sorted(range(t.dim()), key=lambda d: t.stride(d)):
        if t.size(d) == 1:
            continue
        if t.stride(d) != expected:
            return False
        expected *= t.size(d)
    return True


def _flat_view(t: torch.Tensor) -> torch.Tensor:
    """1-D view of a dense tensor in its PHYSICAL order (e.g. NHWC for channels_last)."""
    if t.is_contiguous():
        return t.reshape(-1)
    if not is_dense(t):
        raise ValueError("bucket tensors must be non-overlapping and dense")
    perm = sorted(range(t.dim()), key=lambda d: -t.stride(d))
    return t.permute(*perm).reshape(-1)


def bucket_pack(tensors: Sequence[torch.Tensor], flat: torch.Tensor, offsets: Sequence[int], scale: float = 1.0):
    for t, off in zip(tensors, offsets):
        n = t.numel()
        v = _flat_view(t)
        flat[off:off + n].copy_(v.to(flat.dtype).mul(scale) if scale != 1.0 else v)


def bucket_unpack(tensors: Sequence[torch.Tensor], flat: torch.Tensor, offsets: Sequence[int], scale: float = 1.0):
    for t, off in zip(tensors, offsets):
        n = t.numel()
        src = flat[off:off + n]
        if scale != 1.0:
            src = src.to(torch.promote_types(src.dtype, torch.float32)).mul(scale)
        if t.is_contiguous():
            t.view(-1).copy_(src)
        else:
            perm = sorted(range(t.dim()), key=lambda d: -t.stride(d))
            t.permute(*perm).copy_(src.view([t.shape[d] for d in perm]))


def sgd_step(master, grad, mom, model, *, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
             first_step=False, grad_scale=1.0, dscale: Optional[torch.Tensor] = None):
    g = grad.to(torch.float32) * grad_scale
    if dscale is not None:
        g = g * dscale[0]
    if weight_decay:
        g = g + weight_decay * master
    if momentum:
        if first_step:
            mom.copy_(g)
        else:
            mom.mul_(momentum).add_(g, alpha=1.0 - dampening)
        g = g + momentum * mom if nesterov else mom
    master.add_(g, alpha=-lr)
    if model is not None:
        model.copy_(master)


def adam_step(master, grad, m1, m2, model, *, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, adamw=True,
              step=1, grad_scale=1.0, dscale: Optional[torch.Tensor] = None):
    g = grad.to(torch.float32) * grad_scale
    if dscale is not None:
        g = g * dscale[0]
    if weight_decay and not adamw:
        g = g + weight_decay * master
    if weight_decay and adamw:
        master.mul_(1.0 - lr * weight_decay)
    m1.mul_(beta1).add_(g, alpha=1.0 - beta1)
    m2.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    denom = m2.sqrt() / math.sqrt(bc2) + eps
    master.addcdiv_(m1, denom, value=-lr / bc1)
    if model is not None:
        model.copy_(master)


def grad_norm(flats: Sequence[torch.Tensor], max_norm: float = 0.0, scale: float = 1.0) -> torch.Tensor:
    sq = sum(float((f.to(torch.float32) * scale).pow(2).sum()) for f in flats)
    norm = math.sqrt(sq)
    coef = 1.0
    if max_norm > 0:
        coef = min(1.0, max_norm / (norm + 1e-6))
    return torch.tensor([norm, coef], dtype=torch.float32, device=flats[0].device)


def norm(x, weight, bias, eps, rms, residual=None):
    s = x + residual if residual is not None else x
    xf = s.float()
    if rms:
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    else:
        mu = xf.mean(-1, keepdim=True)
        var = (xf - mu).pow(2).mean(-1, keepdim=True)
        y = (xf - mu) * torch.rsqrt(var + eps)
    if weight is not None:
        y = y * weight.float()
    if bias is not None:
        y = y + bias.float()
    y = y.to(x.dtype)
    return (y, s) if residual is not None else y


def batch_norm_act(x, weight, bias, running_mean, running_var, num_batches_tracked=None, *, training, momentum=0.1,
                   eps=1e-5, relu=False, residual=None):
    import torch.nn.functional as F

    if training and num_batches_tracked is not None:
        num_batches_tracked.add_(1)
        if momentum is None:
            momentum = 1.0 / float(num_batches_tracked)
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum if momentum is not None else 0.0,
                     eps)
    if residual is not None:
        y = y + residual
    if relu:
        y = torch.relu(y)
    return y


def cross_entropy(logits, targets, *, shift=False, vocab=None, ignore_index=-100):
    import torch.nn.functional as F

    v = vocab or logits.size(-1)
    if shift:
        logits, targets = logits[:, :-1], targets[:, 1:]
    return F.cross_entropy(logits[..., :v].reshape(-1, v).float(), targets.reshape(-1), ignore_index=ignore_index)


def attention(q, k, v, *, causal=True, scale=None):
    """[B, S, H, D] / [B, S, Hkv, D] -> [B, S, H, D] via SDPA (fp32 oracle when given fp32)."""
    import torch.nn.functional as F

    h, hkv = q.size(2), k.size(2)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                       is_causal=causal, scale=scale, enable_gqa=h != hkv)
    return o.transpose(1, 2).contiguous()
