"""K13 3x3 / stride 1 / pad 1 NHWC convolution (madnn/ops/csrc/conv3.hip) against a plain PyTorch
fp32 reference: forward, fused BatchNorm statistics, data gradient (same kernel on the flipped
weight) and the autograd path the ResNet models take."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ops():
    from madnn import ops

    assert ops.load_kernels(), "HIP kernel library failed to load"
    return ops


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


# (N, Ci, Co, H, W): ResNet shapes, a tile spanning image seams, odd sizes, M not a multiple of 256
SHAPES = [(2, 64, 64, 56, 56), (3, 128, 128, 28, 28), (5, 64, 128, 14, 14), (7, 256, 64, 7, 7), (3, 64, 192, 5, 9),
          (1, 128, 64, 3, 3)]


@pytest.mark.parametrize("N,Ci,Co,H,W", SHAPES)
def test_conv3x3_fwd_and_stats(N, Ci, Co, H, W):
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(N * 100 + Ci + W)
    x = _cl(torch.randn(N, Ci, H, W, device="cuda", generator=g).bfloat16())
    w = _cl((torch.randn(Co, Ci, 3, 3, device="cuda", generator=g) * (9 * Ci) ** -0.5).bfloat16())
    assert ops.conv3x3_supported(x, w)
    y, part = torch.ops.madnn.conv3x3_fwd(x, w, True)
    ref = F.conv2d(x.float(), w.float(), None, 1, 1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
    yf = y.float()
    s = part.sum(0)
    torch.testing.assert_close(s[0], yf.sum((0, 2, 3)), atol=1e-2 * yf.numel() ** 0.5, rtol=1e-3)
    torch.testing.assert_close(s[1], (yf * yf).sum((0, 2, 3)), atol=1e-2 * yf.numel() ** 0.5, rtol=1e-3)


def test_conv3x3_exact_small_integers():
    """Small-integer data: every product and sum is exact, so K13 must equal the once-rounded
    reference bit for bit (catches a wrong tap / halo row / channel chunk)."""
    _ops()
    g = torch.Generator(device="cuda").manual_seed(5)
    N, Ci, Co, H, W = 3, 128, 64, 11, 13
    x = _cl(torch.randint(-2, 3, (N, Ci, H, W), device="cuda", generator=g).bfloat16())
    w = _cl(torch.randint(-1, 2, (Co, Ci, 3, 3), device="cuda", generator=g).bfloat16())
    w[:, :, 0, 2] += 1  # asymmetric kernel
    y, _ = torch.ops.madnn.conv3x3_fwd(x, w, False)
    assert torch.equal(y, F.conv2d(x.float(), w.float(), None, 1, 1).bfloat16())


# stride 2 (SD = 2): ResNet-50's three stride-2 3x3 shapes, tiles spanning image seams, tiny images
S2_SHAPES = [(2, 128, 128, 56, 56), (3, 256, 256, 28, 28), (4, 512, 512, 14, 14), (5, 64, 128, 8, 6),
             (3, 64, 64, 2, 2)]


@pytest.mark.parametrize("N,Ci,Co,H,W", S2_SHAPES)
def test_conv3x3_stride2_fwd_and_stats(N, Ci, Co, H, W):
    _ops()
    g = torch.Generator(device="cuda").manual_seed(N * 10 + Ci + W)
    x = _cl(torch.randn(N, Ci, H, W, device="cuda", generator=g).bfloat16())
    w = _cl((torch.randn(Co, Ci, 3, 3, device="cuda", generator=g) * (9 * Ci) ** -0.5).bfloat16())
    y, part = torch.ops.madnn.conv3x3_fwd_s2(x, w, True)
    ref = F.conv2d(x.float(), w.float(), None, 2, 1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
    yf = y.float()
    s = part.sum(0)
    torch.testing.assert_close(s[0], yf.sum((0, 2, 3)), atol=1e-2 * yf.numel() ** 0.5, rtol=1e-3)
    torch.testing.assert_close(s[1], (yf * yf).sum((0, 2, 3)), atol=1e-2 * yf.numel() ** 0.5, rtol=1e-3)


def test_conv3x3_stride2_exact_small_integers():
    """Exact integer arithmetic: the stride-2 taps / halo rows / image seams bit for bit."""
    _ops()
    g = torch.Generator(device="cuda").manual_seed(6)
    N, Ci, Co, H, W = 3, 128, 64, 12, 10
    x = _cl(torch.randint(-2, 3, (N, Ci, H, W), device="cuda", generator=g).bfloat16())
    w = _cl(torch.randint(-1, 2, (Co, Ci, 3, 3), device="cuda", generator=g).bfloat16())
    w[:, :, 2, 0] += 1  # asymmetric kernel
    y, _ = torch.ops.madnn.conv3x3_fwd_s2(x, w, False)
    assert torch.equal(y, F.conv2d(x.float(), w.float(), None, 2, 1).bfloat16())


def test_conv3x3_stride2_module_path_autograd():
    """FusedConv2d(stride 2) on a 14x14 map routes its forward to K13's stride-2 kernel (statistics
    included); output, dx and dw match an fp32 nn.Conv2d."""
    ops = _ops()
    from madnn.nn.conv import FusedConv2d

    torch.manual_seed(7)
    conv = FusedConv2d(128, 128, 3, stride=2, padding=1, bias=False).cuda().bfloat16()
    conv = conv.to(memory_format=torch.channels_last)
    x = _cl(torch.randn(4, 128, 14, 14, device="cuda").bfloat16()).requires_grad_(True)
    assert conv._k13s2(x) and ops.conv3x3_s2_supported(x, conv.weight)
    y, part = conv(x, stats=True)
    assert part is not None and part.shape[1:] == (2, 128)
    g = torch.randn_like(y)
    y.backward(g)
    xf = x.detach().float().requires_grad_(True)
    wf = conv.weight.detach().float().requires_grad_(True)
    ref = F.conv2d(xf, wf, None, 2, 1)
    ref.backward(g.float())
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
    for a, b in ((x.grad, xf.grad), (conv.weight.grad, wf.grad)):
        assert float((a.float() - b).norm() / b.norm()) < 1e-2


@pytest.mark.parametrize("N,Ci,Co,H,W", [(2, 64, 64, 56, 56), (3, 128, 64, 14, 14), (2, 64, 128, 7, 9)])
def test_conv3x3_autograd(N, Ci, Co, H, W):
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(Ci + Co + H)
    x = _cl(torch.randn(N, Ci, H, W, device="cuda", generator=g).bfloat16()).requires_grad_(True)
    w = _cl((torch.randn(Co, Ci, 3, 3, device="cuda", generator=g) * (9 * Ci) ** -0.5).bfloat16()).requires_grad_(True)
    dy = _cl(torch.randn(N, Co, H, W, device="cuda", generator=g).bfloat16())
    y, part = ops.conv3x3(x, w, stats=True)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    F.conv2d(xr, wr, None, 1, 1).backward(dy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=0.5, rtol=3e-2)


def test_resnet_block_uses_k13():
    """A ResNet-50 bottleneck in training mode runs its 3x3 on K13 and matches an fp32 copy."""
    _ops()
    from madnn.models.resnet import Bottleneck

    torch.manual_seed(0)
    blk = Bottleneck(256, 64).cuda()
    ref = Bottleneck(256, 64).cuda()
    ref.load_state_dict(blk.state_dict())
    blk = blk.to(torch.bfloat16, memory_format=torch.channels_last)
    for m in blk.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.float()
    assert "K13" in repr(blk.conv2)
    x = _cl(torch.randn(4, 256, 14, 14, device="cuda"))
    y = blk(x.bfloat16())
    yr = ref(x)
    torch.testing.assert_close(y.float(), yr, atol=0.1, rtol=0.05)


@pytest.mark.parametrize("N,Ci,Co,H,W", [(2, 64, 64, 56, 56), (3, 128, 128, 28, 28), (4, 256, 64, 14, 14),
                                          (5, 64, 128, 7, 7), (2, 64, 64, 5, 9)])
def test_conv3x3_wgrad(N, Ci, Co, H, W):
    _ops()
    g = torch.Generator(device="cuda").manual_seed(N + Ci * 3 + W)
    x = _cl(torch.randn(N, Ci, H, W, device="cuda", generator=g).bfloat16())
    dy = _cl(torch.randn(N, Co, H, W, device="cuda", generator=g).bfloat16())
    dw = torch.ops.madnn.conv3x3_wgrad(dy, x, False)
    assert dw.shape == (Co, Ci, 3, 3) and dw.dtype == torch.float32
    assert dw.is_contiguous(memory_format=torch.channels_last)
    xr = x.float().requires_grad_(True)
    wr = torch.zeros(Co, Ci, 3, 3, device="cuda", requires_grad=True)
    F.conv2d(xr, wr, None, 1, 1).backward(dy.float())
    torch.testing.assert_close(dw, wr.grad, atol=2e-3 * (N * H * W) ** 0.5, rtol=1e-3)
    dwb = torch.ops.madnn.conv3x3_wgrad(dy, x, True)
    assert dwb.dtype == torch.bfloat16
    torch.testing.assert_close(dwb.float(), dw, atol=1e-2 * float(dw.abs().max()), rtol=1e-2)


def test_conv3x3_wgrad_exact_small_integers():
    _ops()
    g = torch.Generator(device="cuda").manual_seed(9)
    N, Ci, Co, H, W = 2, 64, 128, 6, 10
    x = _cl(torch.randint(-2, 3, (N, Ci, H, W), device="cuda", generator=g).bfloat16())
    dy = _cl(torch.randint(-2, 3, (N, Co, H, W), device="cuda", generator=g).bfloat16())
    dw = torch.ops.madnn.conv3x3_wgrad(dy, x, False)
    xr = x.float().requires_grad_(True)
    wr = torch.zeros(Co, Ci, 3, 3, device="cuda", requires_grad=True)
    F.conv2d(xr, wr, None, 1, 1).backward(dy.float())
    assert torch.equal(dw, wr.grad)
