"""K10: the ResNet stem convolution (7x7, stride 2, pad 3, 3 -> 64 channels, NHWC bf16) on MFMA vs
fp32 PyTorch references of the same op — forward, the fused BatchNorm statistics, the weight
gradient, and the ResNet stem module that uses them."""
import pytest
import torch
import torch.nn.functional as F

from madnn import ops

pytestmark = pytest.mark.gpu

# (N, H, W): the ImageNet shape, Wo not a multiple of 16 (padded MFMA reduction), odd heights,
# one workgroup owning rows of two images, a batch smaller than the workgroup count
SHAPES = [(2, 224, 224), (3, 33, 48), (1, 64, 64), (5, 17, 24), (2, 224, 8), (1, 7, 256)]


def _img(shape, dev):
    return torch.randn(shape, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)


def _close(a, b, rel):
    torch.testing.assert_close(a, b, atol=rel * b.abs().max().item() + 1e-6, rtol=rel)


@pytest.mark.parametrize("shape", SHAPES)
def test_stem_fwd_stats_wgrad_match_fp32(cuda, shape):
    n, h, w = shape
    torch.manual_seed(0)
    x = _img((n, 3, h, w), cuda)
    wt = (torch.randn(64, 3, 7, 7, device=cuda) * 0.1).bfloat16()
    assert ops.stem_supported(x, wt)
    y, part = torch.ops.madnn.stem_fwd(x, ops._stem_pack(wt), True)
    yr = F.conv2d(x.float(), wt.float(), stride=2, padding=3)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    _close(y.float(), yr, 1e-2)
    yf = y.double().permute(0, 2, 3, 1).reshape(-1, 64)
    tol = 1e-5 * yf.abs().sum(0).max().item() + 1e-6
    torch.testing.assert_close(part[:, 0].double().sum(0), yf.sum(0), atol=tol, rtol=1e-5)
    torch.testing.assert_close(part[:, 1].double().sum(0), (yf * yf).sum(0), atol=tol, rtol=1e-5)

    dy = _img(tuple(yr.shape), cuda)
    dw = torch.ops.madnn.stem_wgrad(dy, x)
    xr = x.float().requires_grad_(False)
    wr = wt.float().requires_grad_(True)
    F.conv2d(xr, wr, stride=2, padding=3).backward(dy.float())
    assert dw.shape == (64, 3, 7, 7) and dw.dtype == torch.float32
    _close(dw, wr.grad, 2e-3)


def test_stem_wgrad_asymmetric(cuda):
    """A one-hot dy at a single pixel and channel picks out one 7x7x3 input patch: catches a
    transposed or shifted (kh, kw, c) order in the weight gradient."""
    x = (torch.arange(1 * 3 * 32 * 32, device=cuda, dtype=torch.float32).reshape(1, 32, 32, 3) % 29 - 14)
    x = x.permute(0, 3, 1, 2).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.zeros(1, 64, 16, 16, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    dy[0, 5, 4, 7] = 1.0
    dw = torch.ops.madnn.stem_wgrad(dy, x)
    xp = F.pad(x.float(), (3, 3, 3, 3))
    patch = xp[0, :, 8:15, 14:21]
    torch.testing.assert_close(dw[5], patch, atol=0, rtol=0)
    assert dw[torch.arange(64, device=cuda) != 5].abs().max().item() == 0


def test_stem_module_autograd_and_bn(cuda):
    from madnn.nn import FusedBatchNorm2d
    from madnn.nn.conv import FusedConv2d

    torch.manual_seed(1)
    conv = FusedConv2d(3, 64, 7, stride=2, padding=3, bias=False).to(cuda).bfloat16()
    bn = FusedBatchNorm2d(64).to(cuda)
    ref_conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(cuda)
    ref_conv.weight.data.copy_(conv.weight.float())
    ref_bn = torch.nn.BatchNorm2d(64).to(cuda)
    x = _img((4, 3, 64, 64), cuda)
    y, st = conv(x, stats=True)
    assert st is not None and "K10" in conv.extra_repr()
    out = bn(y, relu=True, stats=st)
    ref = F.relu(ref_bn(ref_conv(x.float())))
    _close(out.float(), ref, 3e-2)
    g = torch.randn_like(ref)
    out.float().backward(g)
    ref.backward(g)
    _close(conv.weight.grad.float(), ref_conv.weight.grad, 5e-2)
