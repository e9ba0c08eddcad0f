"""ResNet (v1.5, torchvision layout and parameter names) — in-repo because
torchvision is not installed.  BASELINE config 2:
"ResNet-50 auto data-parallel bf16 on 8xMI355X".

The bottleneck 1x1 convolutions (stride 1) run on madnn's K9 MFMA GEMM kernels,
which also compute the following BatchNorm's batch statistics in their epilogue; the stride-1
3x3 convolutions run on K13 (MFMA implicit GEMM over an LDS-staged input halo, statistics in the
epilogue, data grad on the flipped weight); the stride-2 3x3 on the 14x14 map runs its forward on
K13's stride-2 variant (statistics in the epilogue), the larger stride-2 3x3s on MIOpen / CK through
PyTorch-ROCm (a committed per-shape A/B: profiles/r5_conv3x3_s2_ab.json); the 7x7 stem runs on K10 (MFMA
forward with the BatchNorm statistics in its epilogue, MFMA weight gradient); the stem max-pool is madnn's
NHWC kernel (K7, byte argmax + gather backward); every
BatchNorm is madnn's fused NHWC kernel (K5) with the following ReLU and, at the
end of each block, the residual add folded in: ``relu(bn3(conv3(h)) + idt)`` is
one kernel forward and one backward.  The network runs channels_last (NHWC) in
bf16 with fp32 BatchNorm parameters — the layout MIOpen's gfx950 implicit-GEMM
convolutions prefer.
"""
from __future__ import annotations

import os
from typing import List, Optional, Type

import torch
from torch import nn

from ..nn.conv import FusedConv2d
from ..nn.norm import FusedBatchNorm2d as BN
from ..nn.norm import FusedGlobalAvgPool2d, FusedMaxPool2d
from ..ops import (batch_norm_add_bn_relu, bn_relu_conv1x1, bn_relu_conv1x1_epi_supported,
                   bn_relu_conv3x3, conv1x1_route,
                   bn_relu_conv3x3_supported, bn_relu_maxpool, bn_relu_maxpool_supported)

# A/B knob: sum the downsample path's input gradient inside conv1's data grad (1) or by autograd (0)
_FORK_DS = os.environ.get("MADNN_FORK_DOWNSAMPLE", "1") != "0"
# A/B knob: the downsample path's BatchNorm runs inside bn3's kernels (1) or as its own passes (0)
_DUAL_BN = os.environ.get("MADNN_DUAL_BN", "1") != "0"
# A/B knob: the stride-2 1x1 downsample convolution as a stride-1 1x1 on conv1's compact subsample
# of the block input (1) or as a stride-2 library convolution on the full input (0)
_DS_SUB = os.environ.get("MADNN_DS_SUB", "1") != "0"


def conv3x3(cin, cout, stride=1, groups=1, dilation=1):
    # stride 1 runs on K13 (forward + BN statistics, data grad); stride 2 on MIOpen
    return FusedConv2d(cin, cout, 3, stride=stride, padding=dilation, groups=groups, bias=False, dilation=dilation)


def conv1x1(cin, cout, stride=1):
    return FusedConv2d(cin, cout, 1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = BN(planes)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = BN(planes)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y, st = self.conv1(x, stats=True)
        out = self.bn1(y, relu=True, stats=st)
        y, st = self.conv2(out, stats=True)
        return self.bn2(y, residual=idt, relu=True, stats=st)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = BN(planes)
        self.conv2 = conv3x3(planes, planes, stride)   # stride on the 3x3 (v1.5)
        self.bn2 = BN(planes)
        self.conv3 = conv1x1(planes, planes * 4)
        self.bn3 = BN(planes * 4)
        self.downsample = downsample

    def forward(self, x):
        if self.downsample is None:
            # K9: BN statistics from the GEMM epilogue; the identity path's gradient is added
            # inside conv1's data-grad kernel (no separate residual-gradient add)
            y, st, idt = self.conv1(x, stats=True, fork=True)
            if isinstance(idt, torch.Tensor) and isinstance(self.bn3, BN) and self.conv1._k9(x) \
                    and conv1x1_route(x.size(1), self.conv1.weight.size(0))[1] == "k9":
                # idt's only consumer is bn3 and its gradient is summed inside K9's data grad: that
                # kernel applies bn3's ReLU mask itself (ops._BNFn deferred mask)
                idt._madnn_defer_mask = True
        elif _FORK_DS:
            # the downsample path's input gradient is likewise summed inside conv1's data grad
            dual = self._dual_bn()
            sub = dual and _DS_SUB and isinstance(x, torch.Tensor) and self.downsample[0].subsampled_ok()
            y, st, xf = self.conv1(x, stats=True, fork=2 if sub else True)
            if dual:
                # relu(bn3(conv3) + bn_ds(conv_ds)): the downsample BN is applied inside bn3's
                # passes (forward and backward), its normalised output never written to HBM.
                # sub: conv1 hands over the compact x[:, :, ::2, ::2] and the stride-2 downsample
                # runs as a stride-1 1x1 on it (K9, BN statistics from its epilogue); its compact
                # input gradient is added into conv1's data grad at the even pixels
                yd, std = (self.downsample[0].forward_subsampled(xf, stats=True) if sub
                           else self.downsample[0](xf, stats=True))
                y, st = self._bn1_conv2(y, st)
                y, st = self._bn2_conv3(y, st)
                return batch_norm_add_bn_relu(y, yd, self.bn3, self.downsample[1], st, std)
            idt = self.downsample(xf)
        else:
            idt = self.downsample(x)
            y, st = self.conv1(x, stats=True)
        y, st = self._bn1_conv2(y, st)   # K13 at stride 1: BN statistics from the epilogue
        y, st = self._bn2_conv3(y, st)
        return self.bn3(y, residual=idt, relu=True, stats=st)   # relu(bn3 + idt): one kernel

    def _bn1_conv2(self, y, st):
        """conv2(relu(bn1(y))): with conv2 on K13, bn1's backward reduction is taken in conv2's
        data-grad epilogue (ops.bn_relu_conv3x3); the stride-2 conv2s take the module path (K13's stride-2
        forward on small maps, the library otherwise)."""
        if isinstance(y, torch.Tensor) and isinstance(self.bn1, BN) and isinstance(self.conv2, FusedConv2d) \
                and self.conv2._k13(y) \
                and bn_relu_conv3x3_supported(y, self.bn1, self.conv2.weight):
            return bn_relu_conv3x3(y, self.bn1, self.conv2.weight, stats_in=st, stats=True)
        out = self.bn1(y, relu=True, stats=st)
        return self.conv2(out, stats=True)

    def _bn2_conv3(self, y, st):
        """conv3(relu(bn2(y))): when conv3's data grad runs on K9, bn2's backward reduction is taken
        in that kernel's epilogue."""
        if isinstance(y, torch.Tensor) and isinstance(self.bn2, BN) and isinstance(self.conv3, FusedConv2d) \
                and self.conv3._k9(y) and bn_relu_conv1x1_epi_supported(y, self.bn2, self.conv3.weight):
            return bn_relu_conv1x1(y, self.bn2, self.conv3.weight, stats_in=st, stats=True)
        out = self.bn2(y, relu=True, stats=st)
        return self.conv3(out, stats=True)

    def _dual_bn(self) -> bool:
        ds = self.downsample
        return (_DUAL_BN and isinstance(ds, nn.Sequential) and len(ds) == 2
                and isinstance(ds[0], FusedConv2d) and isinstance(ds[1], BN) and isinstance(self.bn3, BN))


class ResNet(nn.Module):
    def __init__(self, block: Type[nn.Module], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = True, width: int = 64):
        super().__init__()
        self.inplanes = width
        self.conv1 = FusedConv2d(3, width, 7, stride=2, padding=3, bias=False)   # K10 stem
        self.bn1 = BN(width)
        self.maxpool = FusedMaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, width, layers[0])
        self.layer2 = self._make_layer(block, width * 2, layers[1], stride=2)
        self.layer3 = self._make_layer(block, width * 4, layers[2], stride=2)
        self.layer4 = self._make_layer(block, width * 8, layers[3], stride=2)
        self.avgpool = FusedGlobalAvgPool2d((1, 1))
        self.fc = nn.Linear(width * 8 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):  # FusedBatchNorm2d included
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       BN(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def stem(self, x):
        y, st = self.conv1(x, stats=True)
        if isinstance(self.bn1, BN) and isinstance(self.maxpool, FusedMaxPool2d) \
                and bn_relu_maxpool_supported(y, self.bn1, self.maxpool):
            # BN apply + ReLU inside the max-pool's window loads; the pool gradient gathered
            # inside the BN backward: relu(bn1(y)) and its gradient never reach HBM
            return bn_relu_maxpool(y, self.bn1, self.maxpool, st)
        return self.maxpool(self.bn1(y, relu=True, stats=st))

    def head(self, x):
        return self.fc(torch.flatten(self.avgpool(x), 1))

    def forward(self, x):
        x = self.layer4(self.layer3(self.layer2(self.layer1(self.stem(x)))))
        return self.head(x)

    def pipeline_layers(self):
        """The spine the planner costs / partitions: stem, every residual block, head."""
        blocks = [b for layer in (self.layer1, self.layer2, self.layer3, self.layer4) for b in layer]
        return [_Bound(self, "stem"), *blocks, _Bound(self, "head")]


class _Bound(nn.Module):
    """One single-tensor piece of a model's forward as a layer (shares the model's modules)."""

    def __init__(self, model: nn.Module, method: str):
        super().__init__()
        self.parts = nn.ModuleDict({n: m for n, m in model.named_children()
                                    if n in {"stem": ("conv1", "bn1", "maxpool"),
                                             "head": ("avgpool", "fc")}[method]})
        object.__setattr__(self, "_model", model)
        self.method = method

    def forward(self, x):
        return getattr(self._model, self.method)(x)


def resnet18(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, **kw)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, **kw)


def resnet101(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes, **kw)
