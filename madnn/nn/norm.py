"""LayerNorm / RMSNorm modules backed by the gfx950 K3 kernel.

Drop-in for ``nn.LayerNorm`` (same parameter names ``weight``/``bias``, so
state dicts interchange).  On HIP tensors they call ``madnn.ops.layer_norm`` /
``rms_norm`` (one fused kernel each way, optional fused residual add); on CPU
the eager reference.  ``swap_layernorms(model)`` replaces every eligible
``nn.LayerNorm`` of an arbitrary model in place; ``distribute()`` does this (and
more) through :func:`madnn.nn.swap.use_madnn_kernels`.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from .. import ops


class FusedLayerNorm(nn.Module):
    def __init__(self, normalized_shape, eps: float = 1e-5, elementwise_affine: bool = True, bias: bool = True,
                 device=None, dtype=None):
        super().__init__()
        if isinstance(normalized_shape, int):
            normalized_shape = (normalized_shape,)
        self.normalized_shape = tuple(normalized_shape)
        if len(self.normalized_shape) != 1:
            raise ValueError("FusedLayerNorm normalises the last dimension only")
        self.eps = eps
        h = self.normalized_shape[0]
        self.weight = nn.Parameter(torch.ones(h, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.zeros(h, device=device, dtype=dtype)) if bias else None

    def reset_parameters(self):
        with torch.no_grad():
            self.weight.fill_(1.0)
            if self.bias is not None:
                self.bias.zero_()

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, fork: bool = False):
        """LN(x); with ``residual``, (LN(x + residual), x + residual) in one kernel; with ``fork``,
        (LN(x), x) whose second output's gradient joins x's inside the LN backward pass."""
        if residual is not None and residual.dtype != x.dtype:
            residual = residual.to(x.dtype)
        return ops.layer_norm(x, self.weight, self.bias, self.eps, residual=residual, fork=fork)

    def extra_repr(self):
        return f"{self.normalized_shape}, eps={self.eps}, kernel=madnn.K3"


class FusedRMSNorm(nn.Module):
    def __init__(self, hidden: int, eps: float = 1e-6, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hidden, device=device, dtype=dtype))

    def reset_parameters(self):
        with torch.no_grad():
            self.weight.fill_(1.0)

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, fork: bool = False):
        if residual is not None and residual.dtype != x.dtype:
            residual = residual.to(x.dtype)
        return ops.rms_norm(x, self.weight, self.eps, residual=residual, fork=fork)

    def extra_repr(self):
        return f"{self.weight.numel()}, eps={self.eps}, kernel=madnn.K3"


def swap_layernorms(model: nn.Module) -> int:
    """Replace eligible ``nn.LayerNorm`` modules by :class:`FusedLayerNorm` (weights kept)."""
    n = 0
    for name, child in list(model.named_children()):
        if type(child) is nn.LayerNorm and len(child.normalized_shape) == 1 and child.elementwise_affine \
                and ops.hidden_supported(child.normalized_shape[0]):
            new = FusedLayerNorm(child.normalized_shape, child.eps, bias=child.bias is not None,
                                 device=child.weight.device, dtype=child.weight.dtype)
            with torch.no_grad():
                new.weight.copy_(child.weight)
                if child.bias is not None:
                    new.bias.copy_(child.bias)
            setattr(model, name, new)
            n += 1
        else:
            n += swap_layernorms(child)
    return n


class FusedBatchNorm2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` whose forward optionally fuses a residual add and a ReLU:
    ``act(BN(x) + residual)``; NHWC (channels_last) HIP tensors run the K5 kernel,
    everything else the eager composition.  Same parameters/buffers as
    ``nn.BatchNorm2d`` (state dicts interchange; ``isinstance`` holds)."""

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, relu: bool = False,
                stats: Optional[torch.Tensor] = None):
        """``stats``: partial batch statistics of ``x`` from the producing kernel
        (:class:`~madnn.nn.FusedConv2d` with ``stats=True``), or None."""
        training = self.training or not self.track_running_stats
        return ops.batch_norm_act(x, self.weight, self.bias,
                                  self.running_mean if (not self.training or self.track_running_stats) else None,
                                  self.running_var if (not self.training or self.track_running_stats) else None,
                                  self.num_batches_tracked if (self.training and self.track_running_stats) else None,
                                  training=training, momentum=self.momentum, eps=self.eps, relu=relu,
                                  residual=residual, stats=stats)


class FusedMaxPool2d(nn.MaxPool2d):
    """``nn.MaxPool2d`` whose NHWC (channels_last) HIP path is the K7 kernel pair:
    a byte-per-element argmax instead of int64 indices and a gather backward
    (no dx memset, no scatter).  Any other input falls back to ``F.max_pool2d``."""

    def forward(self, x: torch.Tensor):
        if self.return_indices:
            return super().forward(x)
        return ops.max_pool2d(x, self.kernel_size, self.stride, self.padding, self.dilation, self.ceil_mode)


class _GlobalAvgPool(torch.autograd.Function):
    """mean over H, W.  Backward writes dx = dy/(H*W) broadcast in ONE pass straight into the
    input's memory format; ATen's AdaptiveAvgPool2d backward on a channels_last input ran an
    NCHW-strided expand plus a slow strided layout copy (188 us/step on ResNet-50 batch 512,
    profiles/r1_resnet50_dp1_pool.md) in front of the first BatchNorm backward."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        ctx.cl = x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()
        return x.mean((2, 3), keepdim=True)

    @staticmethod
    def backward(ctx, g):
        n, c, h, w = ctx.shape
        g = (g.reshape(n, c).float() * (1.0 / (h * w))).to(g.dtype)
        if ctx.cl:
            return g.view(n, 1, 1, c).expand(n, h, w, c).contiguous().permute(0, 3, 1, 2)
        return g.view(n, c, 1, 1).expand(n, c, h, w).contiguous()


class FusedGlobalAvgPool2d(nn.AdaptiveAvgPool2d):
    """``nn.AdaptiveAvgPool2d((1, 1))`` with a single-pass, memory-format-preserving backward."""

    def __init__(self, output_size=(1, 1)):
        super().__init__(output_size)

    def forward(self, x: torch.Tensor):
        os_ = self.output_size
        if x.dim() == 4 and (os_ == 1 or tuple(os_) == (1, 1)):
            return _GlobalAvgPool.apply(x)
        return super().forward(x)
