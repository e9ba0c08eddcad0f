"""Convolution module backed by madnn's gfx950 K9 kernels.

``FusedConv2d`` is a drop-in ``nn.Conv2d`` (same parameters, state dict and
``isinstance``).  A stride-1, unpadded, ungrouped, bias-free 1x1 convolution of an
NHWC (channels_last) bf16 HIP tensor runs as three MFMA GEMMs (``madnn.ops.conv1x1``:
forward, data grad, weight grad) and can hand the following
:class:`~madnn.nn.FusedBatchNorm2d` its batch statistics, computed in the GEMM
epilogue, so the BatchNorm skips its statistics pass.  Every other configuration runs
``nn.Conv2d`` (MIOpen on the GPU), except the ResNet stem (7x7, stride 2, pad 3, 3 -> 64
channels), which runs on K10 (``madnn.ops.stem_conv``, also with the BatchNorm statistics), and
3x3 / stride 1 / pad 1 convolutions with channel counts that are multiples of 64, which run on K13
(``madnn.ops.conv3x3``: forward with the statistics, data grad; weight grad on MIOpen or K13), and
3x3 / stride 2 ones on small maps (``madnn.ops.conv3x3_s2``: K13 forward with the statistics).
``MADNN_CONV1X1=0`` / ``MADNN_STEM=0`` / ``MADNN_CONV3X3=0`` disable the K9 / K10 / K13 paths
(A/B runs).
"""
from __future__ import annotations

import os

import torch
from torch import nn

from .. import ops

_K9 = os.environ.get("MADNN_CONV1X1", "1") != "0"


class FusedConv2d(nn.Conv2d):
    def _k9(self, x: torch.Tensor) -> bool:
        return (_K9 and self.kernel_size == (1, 1) and self.stride == (1, 1) and self.dilation == (1, 1)
                and self.groups == 1 and self.bias is None and self.padding in ((0, 0), "valid")
                and ops.conv1x1_supported(x, self.weight))

    def _k13(self, x: torch.Tensor) -> bool:
        return (self.kernel_size == (3, 3) and self.stride == (1, 1) and self.padding == (1, 1)
                and self.dilation == (1, 1) and self.groups == 1 and self.bias is None
                and self.padding_mode == "zeros" and ops.conv3x3_supported(x, self.weight))

    def _k13s2(self, x: torch.Tensor) -> bool:
        return (self.kernel_size == (3, 3) and self.stride == (2, 2) and self.padding == (1, 1)
                and self.dilation == (1, 1) and self.groups == 1 and self.bias is None
                and self.padding_mode == "zeros" and ops.conv3x3_s2_supported(x, self.weight))

    def _k10(self, x: torch.Tensor) -> bool:
        return (self.kernel_size == (7, 7) and self.stride == (2, 2) and self.padding == (3, 3)
                and self.dilation == (1, 1) and self.groups == 1 and self.bias is None
                and ops.stem_supported(x, self.weight))

    def forward(self, x: torch.Tensor, stats: bool = False, fork: bool = False):
        """``conv(x)``.  ``stats=True`` also returns ``partial``, the batch statistics of ``y`` for
        :class:`~madnn.nn.FusedBatchNorm2d` (None when not computed by the kernel); ``fork=True``
        also returns ``x`` for use as a residual path -- on the K9 path its gradient is summed
        inside this convolution's data-grad kernel instead of by a separate add."""
        if self._k9(x):
            return ops.conv1x1(x, self.weight, stats=stats, fork=fork)
        if not fork and self._k13(x):
            return ops.conv3x3(x, self.weight, stats=stats)
        if not fork and self._k13s2(x):
            return ops.conv3x3_s2(x, self.weight, stats=stats)
        if not fork and self._k10(x):
            return ops.stem_conv(x, self.weight, stats=stats)
        out = [super().forward(x)]
        if stats:
            out.append(None)
        if fork:
            out.append(x[:, :, ::2, ::2] if fork == 2 else x)
        return out[0] if len(out) == 1 else tuple(out)

    def subsampled_ok(self) -> bool:
        """A 1x1 / stride-2 / unpadded convolution: equal to a stride-1 1x1 on ``x[:, :, ::2, ::2]``."""
        return (self.kernel_size == (1, 1) and self.stride == (2, 2) and self.padding in ((0, 0), "valid")
                and self.dilation == (1, 1) and self.groups == 1 and self.bias is None)

    def forward_subsampled(self, xs: torch.Tensor, stats: bool = False):
        """This stride-2 1x1 convolution given the subsampled input ``xs = x[:, :, ::2, ::2]`` (e.g. from
        ``conv1x1(..., fork=2)``): a stride-1 1x1 on K9 / the library (with the statistics when on K9)."""
        if _K9 and ops.conv1x1_supported(xs, self.weight):
            return ops.conv1x1(xs, self.weight, stats=stats)
        y = torch.nn.functional.conv2d(xs, self.weight)
        return (y, None) if stats else y

    def extra_repr(self):
        k = {(1, 1): ", kernel=madnn.K9", (7, 7): ", kernel=madnn.K10",
             (3, 3): ", kernel=madnn.K13" if self.stride in ((1, 1), (2, 2)) else ""}.get(self.kernel_size, "")
        return super().extra_repr() + k
