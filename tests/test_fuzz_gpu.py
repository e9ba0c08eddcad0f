"""Shape fuzzing (hypothesis) of the hand-written kernels against their fp32 references: the T2
tier of SURVEY §4.2 ("odd sizes, non-multiples of 64/256, empty tensors").  One process, a bounded
number of examples per kernel, no deadline (the first launch of a kernel compiles nothing but
pays the HIP module load)."""
import pytest
import torch
import torch.nn.functional as F
from hypothesis import HealthCheck, given, settings, strategies as st

from madnn import ops
from madnn.ops import reference as R

pytestmark = pytest.mark.gpu
FUZZ = settings(max_examples=12, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])


@FUZZ
@given(sizes=st.lists(st.integers(0, 5000), min_size=1, max_size=12), scale=st.sampled_from([1.0, 0.5, 0.125]),
       bf16=st.booleans())
def test_fuzz_bucket_roundtrip(cuda, sizes, scale, bf16):
    dt = torch.bfloat16 if bf16 else torch.float32
    ts = [torch.randn(n, device=cuda).to(dt) for n in sizes]
    offs, n = [], 0
    for t in ts:
        offs.append(n)
        n += (t.numel() + 15) // 16 * 16
    flat = torch.zeros(max(n, 16), device=cuda)
    ops.bucket_pack(ts, flat, offs, scale)
    ref = torch.zeros(max(n, 16))
    R.bucket_pack([t.cpu() for t in ts], ref, offs, scale)
    torch.testing.assert_close(flat.cpu(), ref)
    outs = [torch.empty_like(t) for t in ts]
    ops.bucket_unpack(outs, flat, offs, 1.0 / scale)
    for o, t in zip(outs, ts):
        torch.testing.assert_close(o.float(), t.float(), atol=1e-2 if bf16 else 1e-6, rtol=1e-2 if bf16 else 1e-6)


@FUZZ
@given(n=st.integers(0, 300_000), momentum=st.sampled_from([0.0, 0.9]), wd=st.sampled_from([0.0, 1e-2]))
def test_fuzz_sgd(cuda, n, momentum, wd):
    p = torch.randn(n, device=cuda)
    g = torch.randn(n, device=cuda).bfloat16()
    m = torch.randn(n, device=cuda) if momentum else None
    pr, mr = p.cpu().clone(), (m.cpu().clone() if m is not None else None)
    ops.sgd_step(p, g, m, None, lr=0.05, momentum=momentum, weight_decay=wd, first_step=False)
    R.sgd_step(pr, g.cpu(), mr, None, lr=0.05, momentum=momentum, weight_decay=wd, first_step=False)
    torch.testing.assert_close(p.cpu(), pr, atol=1e-5, rtol=1e-5)


@FUZZ
@given(n=st.integers(0, 300_000), step=st.integers(1, 5))
def test_fuzz_adam(cuda, n, step):
    p = torch.randn(n, device=cuda)
    m1, m2 = torch.randn(n, device=cuda) * 0.1, torch.rand(n, device=cuda) * 0.01
    g = torch.randn(n, device=cuda).bfloat16()
    pr, m1r, m2r = p.cpu().clone(), m1.cpu().clone(), m2.cpu().clone()
    ops.adam_step(p, g, m1, m2, None, lr=1e-3, weight_decay=0.01, step=step)
    R.adam_step(pr, g.cpu(), m1r, m2r, None, lr=1e-3, weight_decay=0.01, step=step)
    torch.testing.assert_close(p.cpu(), pr, atol=1e-5, rtol=1e-5)


@FUZZ
@given(rows=st.integers(1, 700), h8=st.integers(1, 512), rms=st.booleans())
def test_fuzz_norm(cuda, rows, h8, rms):
    H = 8 * h8
    x = torch.randn(rows, H, device=cuda).bfloat16().requires_grad_(True)
    w = (1 + 0.1 * torch.randn(H, device=cuda)).requires_grad_(True)
    b = (0.1 * torch.randn(H, device=cuda)).requires_grad_(True)
    y = ops.rms_norm(x, w, eps=1e-6) if rms else ops.layer_norm(x, w, b, eps=1e-5)
    xr = x.detach().float().requires_grad_(True)
    yr = R.norm(xr, w, None if rms else b, 1e-6 if rms else 1e-5, rms, None)
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)


@FUZZ
@given(m=st.integers(1, 1200), n8=st.integers(1, 96), k64=st.integers(1, 12))
def test_fuzz_k12_linear(cuda, m, n8, k64):
    N, K = 8 * n8, 64 * k64
    x = torch.randn(m, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * K ** -0.5).bfloat16()
    y, _ = torch.ops.madnn.linear_fwd(x, w, None, None, 0, False)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), atol=3e-2, rtol=2e-2)


@FUZZ
@given(nb=st.integers(1, 3), h=st.integers(1, 20), w=st.integers(1, 40), ci=st.sampled_from([64, 128]),
       co=st.sampled_from([64, 128, 192]))
def test_fuzz_k13_conv3x3(cuda, nb, h, w, ci, co):
    x = torch.randn(nb, ci, h, w, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(co, ci, 3, 3, device=cuda) * (9 * ci) ** -0.5).bfloat16().contiguous(
        memory_format=torch.channels_last)
    y, part = torch.ops.madnn.conv3x3_fwd(x, wt, True)
    ref = F.conv2d(x.float(), wt.float(), None, 1, 1)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(part.sum(0)[0], y.float().sum((0, 2, 3)), atol=0.05 * (nb * h * w) ** 0.5, rtol=1e-3)
    dy = torch.randn_like(y)
    dw = torch.ops.madnn.conv3x3_wgrad(dy, x, False)
    xr = x.float().requires_grad_(True)
    wr = torch.zeros(co, ci, 3, 3, device=cuda, requires_grad=True)
    F.conv2d(xr, wr, None, 1, 1).backward(dy.float())
    torch.testing.assert_close(dw, wr.grad, atol=3e-3 * (nb * h * w) ** 0.5, rtol=1e-3)
