"""Numerics of the hand-written gfx950 kernels against fp32 PyTorch references.

Each HIP kernel (K1 FusedSGD, K2 FusedAdam, K3 LayerNorm/RMSNorm, K4 bucket
pack/unpack/scale-cast, grad-norm) is compared with madnn.ops.reference, the
eager fp32 implementation of the same op.  Shapes include odd sizes,
non-multiples of 8/64/256, channels_last tensors and empty tensors.
"""
import math

import pytest
import torch

import madnn
from madnn import ops
from madnn.ops import reference as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("fdt", [torch.float32, torch.bfloat16])
def test_bucket_pack_unpack(cuda, tdt, fdt):
    torch.manual_seed(0)
    shapes = [(7,), (64,), (3, 5), (1000, 3), (2049,), (0,), (33, 17, 5)]
    ts = [torch.randn(s, device=cuda).to(tdt) for s in shapes]
    offs, n = [], 0
    for t in ts:
        offs.append(n)
        n += (t.numel() + 15) // 16 * 16
    flat = torch.zeros(n, device=cuda, dtype=fdt)
    ops.bucket_pack(ts, flat, offs, 0.5)
    ref = torch.zeros(n, dtype=fdt)
    R.bucket_pack([t.cpu() for t in ts], ref, offs, 0.5)
    tol = 1e-2 if torch.bfloat16 in (tdt, fdt) else 1e-6
    torch.testing.assert_close(flat.cpu().float(), ref.float(), atol=tol, rtol=tol)
    outs = [torch.empty_like(t) for t in ts]
    ops.bucket_unpack(outs, flat, offs, 2.0)
    for o, t in zip(outs, ts):
        torch.testing.assert_close(o.float(), t.float(), atol=2 * tol, rtol=2 * tol)


def test_bucket_channels_last_and_many_tensors(cuda):
    torch.manual_seed(1)
    ts = [torch.randn(8, 3 + i % 5, 3, 3, device=cuda).contiguous(memory_format=torch.channels_last)
          for i in range(120)]  # > 48 tensors: multiple launches
    offs, n = [], 0
    for t in ts:
        offs.append(n)
        n += (t.numel() + 15) // 16 * 16
    flat = torch.zeros(n, device=cuda)
    ops.bucket_pack(ts, flat, offs, 1.0)
    ref = torch.zeros(n)
    R.bucket_pack([t.cpu() for t in ts], ref, offs, 1.0)
    torch.testing.assert_close(flat.cpu(), ref)
    outs = [torch.empty_like(t) for t in ts]
    ops.bucket_unpack(outs, flat, offs, 1.0)
    for o, t in zip(outs, ts):
        torch.testing.assert_close(o, t)


def test_flat_scale_cast(cuda):
    x = torch.randn(100003, device=cuda)
    y = torch.empty(100003, device=cuda, dtype=torch.bfloat16)
    ops.flat_scale_cast(x, y, 0.25)
    torch.testing.assert_close(y.float(), (x * 0.25).bfloat16().float())


@pytest.mark.parametrize("n", [1, 31, 4096, 1_000_003])
@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("nesterov", [False, True])
def test_sgd_step(cuda, n, gdt, nesterov):
    torch.manual_seed(2)
    p = torch.randn(n, device=cuda)
    g = torch.randn(n, device=cuda).to(gdt)
    m = torch.randn(n, device=cuda)
    model = torch.empty(n, device=cuda, dtype=torch.bfloat16)
    pr, mr = p.cpu().clone(), m.cpu().clone()
    for first in (True, False):
        ops.sgd_step(p, g, m, model, lr=0.1, momentum=0.9, dampening=0.0, weight_decay=1e-2, nesterov=nesterov,
                     first_step=first, grad_scale=0.5)
        R.sgd_step(pr, g.cpu(), mr, None, lr=0.1, momentum=0.9, dampening=0.0, weight_decay=1e-2,
                   nesterov=nesterov, first_step=first, grad_scale=0.5)
    torch.testing.assert_close(p.cpu(), pr, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(m.cpu(), mr, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(model.float(), p.bfloat16().float())


@pytest.mark.parametrize("n", [5, 4096, 777_777])
@pytest.mark.parametrize("adamw", [True, False])
def test_adam_step(cuda, n, adamw):
    torch.manual_seed(3)
    p = torch.randn(n, device=cuda)
    m1 = torch.zeros(n, device=cuda)
    m2 = torch.zeros(n, device=cuda)
    model = torch.empty(n, device=cuda, dtype=torch.bfloat16)
    pr, m1r, m2r = p.cpu().clone(), m1.cpu().clone(), m2.cpu().clone()
    for step in range(1, 4):
        g = torch.randn(n, device=cuda).bfloat16()
        ops.adam_step(p, g, m1, m2, model, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1,
                      adamw=adamw, step=step, grad_scale=1.0)
        R.adam_step(pr, g.cpu(), m1r, m2r, None, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1,
                    adamw=adamw, step=step)
    torch.testing.assert_close(p.cpu(), pr, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(m1.cpu(), m1r, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(m2.cpu(), m2r, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(model.float(), p.bfloat16().float())


def test_grad_norm_and_device_clip(cuda):
    a = torch.randn(1_000_000, device=cuda)
    b = torch.randn(3333, device=cuda).bfloat16()
    out = ops.grad_norm([a, b], max_norm=1.0)
    ref = math.sqrt(float(a.double().pow(2).sum() + b.double().pow(2).sum()))
    assert abs(float(out[0]) - ref) / ref < 1e-4
    assert abs(float(out[1]) - 1.0 / (ref + 1e-6)) < 1e-6
    # dscale path: the clip coefficient multiplies the gradient inside the SGD kernel
    p = torch.zeros(1_000_000, device=cuda)
    ops.sgd_step(p, a, None, None, lr=1.0, dscale=out[1:2])
    torch.testing.assert_close(p, -a * out[1], atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("H", [64, 768, 1024, 1536, 4096, 8192])
@pytest.mark.parametrize("xdt,wdt", [(torch.bfloat16, torch.float32), (torch.float32, torch.float32),
                                     (torch.bfloat16, torch.bfloat16)])
@pytest.mark.parametrize("rms", [False, True])
def test_norm_fwd_bwd(cuda, H, xdt, wdt, rms):
    torch.manual_seed(4)
    rows = 257
    x = (torch.randn(rows, H, device=cuda) * 2 + 0.5).to(xdt).requires_grad_(True)
    w = (torch.rand(H, device=cuda) + 0.5).to(wdt).requires_grad_(True)
    b = None if rms else (torch.randn(H, device=cuda) * 0.1).to(wdt).requires_grad_(True)
    dy = torch.randn(rows, H, device=cuda).to(xdt)
    y = ops.rms_norm(x, w, eps=1e-6) if rms else ops.layer_norm(x, w, b, eps=1e-5)
    y.backward(dy)
    # fp32 reference of the same op
    xr = x.detach().float().cpu().requires_grad_(True)
    wr = w.detach().float().cpu().requires_grad_(True)
    br = None if rms else b.detach().float().cpu().requires_grad_(True)
    yr = R.norm(xr, wr, br, 1e-6 if rms else 1e-5, rms)
    yr.backward(dy.float().cpu())
    tol = 2e-2 if xdt == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float().cpu(), yr, atol=tol, rtol=tol)
    torch.testing.assert_close(x.grad.float().cpu(), xr.grad, atol=tol * 2, rtol=tol * 2)
    gtol = 5e-2 if (xdt == torch.bfloat16 or wdt == torch.bfloat16) else 1e-3
    torch.testing.assert_close(w.grad.float().cpu(), wr.grad, atol=gtol * math.sqrt(rows), rtol=gtol)
    if not rms:
        torch.testing.assert_close(b.grad.float().cpu(), br.grad, atol=gtol * math.sqrt(rows), rtol=gtol)


def test_norm_fused_residual(cuda):
    torch.manual_seed(5)
    x = torch.randn(4, 33, 1024, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(4, 33, 1024, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    w = torch.rand(1024, device=cuda, requires_grad=True)
    b = torch.randn(1024, device=cuda, requires_grad=True)
    y, s = ops.layer_norm(x, w, b, residual=r)
    (y.float().pow(2).sum() + s.float().sum()).backward()
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    sr = xr + rr
    yr = torch.nn.functional.layer_norm(sr, (1024,), wr, br, 1e-5)
    (yr.pow(2).sum() + sr.sum()).backward()
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=8e-2, rtol=5e-2)
    torch.testing.assert_close(r.grad.float(), rr.grad, atol=8e-2, rtol=5e-2)


def test_norm_large_rows_multi_pass(cuda):
    # rows >> grid cap: every workgroup loops over several rows (grid-stride path)
    x = torch.randn(20000, 1024, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(1024, device=cuda, requires_grad=True)
    b = torch.zeros(1024, device=cuda, requires_grad=True)
    y = ops.layer_norm(x, w, b)
    y.float().sum().backward()
    ref = torch.nn.functional.layer_norm(x.detach().float(), (1024,))
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
    assert torch.isfinite(w.grad).all()


@pytest.mark.parametrize("C", [8, 64, 256, 1000, 2048])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True), (False, True)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_batchnorm_fused_nhwc(cuda, C, relu, res, dt):
    """K5 vs eager fp32 act(BN(x) + residual): outputs, running stats, nbt and all grads."""
    torch.manual_seed(6)
    N, H, W = 4, 7, 5
    x = (torch.randn(N, C, H, W, device=cuda) * 1.5 + 0.3).to(dt).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    r = None
    if res:
        r = torch.randn(N, C, H, W, device=cuda).to(dt).contiguous(memory_format=torch.channels_last)
        r.requires_grad_(True)
    w = (torch.rand(C, device=cuda) + 0.5).requires_grad_(True)
    b = (torch.randn(C, device=cuda) * 0.1).requires_grad_(True)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    nbt = torch.zeros((), dtype=torch.long, device=cuda)
    y = ops.batch_norm_act(x, w, b, rm, rv, nbt, training=True, momentum=0.1, eps=1e-5, relu=relu, residual=r)
    dy = torch.randn_like(y)
    y.backward(dy)
    # fp32 eager reference
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if res else None
    wr = w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    rmr, rvr = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    yr = torch.nn.functional.batch_norm(xr, rmr, rvr, wr, br, True, 0.1, 1e-5)
    if res:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    yr.backward(dy.float())
    tol = 3e-2 if dt == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    torch.testing.assert_close(rm, rmr, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rv, rvr, atol=1e-4, rtol=1e-4)
    assert int(nbt) == 1
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=tol * 3, rtol=tol * 3)
    gt = 0.15 if dt == torch.bfloat16 else 1e-3
    torch.testing.assert_close(w.grad, wr.grad, atol=gt, rtol=gt)
    torch.testing.assert_close(b.grad, br.grad, atol=gt, rtol=gt)
    if res:
        torch.testing.assert_close(r.grad.float(), rr.grad, atol=tol, rtol=tol)


def test_batchnorm_fused_eval_and_large(cuda):
    torch.manual_seed(7)
    C = 256
    x = torch.randn(64, C, 56, 56, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    w, b = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda)
    rm, rv = torch.randn(C, device=cuda), torch.rand(C, device=cuda) + 0.5
    with torch.no_grad():
        y = ops.batch_norm_act(x, w, b, rm, rv, training=False, relu=True)
        yr = torch.relu(torch.nn.functional.batch_norm(x.float(), rm, rv, w, b, False, 0.1, 1e-5))
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    # training stats over 200k rows: exact-ish mean/var vs fp64
    rm2, rv2 = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    ops.batch_norm_act(x, w, b, rm2, rv2, training=True, momentum=1.0)
    xd = x.double().permute(0, 2, 3, 1).reshape(-1, C)
    torch.testing.assert_close(rm2.double(), xd.mean(0), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rv2.double(), xd.var(0, unbiased=True), atol=1e-4, rtol=1e-4)


def test_fused_resnet_block_matches_eager(cuda):
    """A Bottleneck with fused BN vs the same weights through eager nn ops (fp32)."""
    from madnn.models.resnet import Bottleneck

    torch.manual_seed(8)
    blk = Bottleneck(64, 16).to(cuda)
    for m in blk.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(m.weight, 0.5, 1.5)
    x = torch.randn(8, 64, 14, 14, device=cuda).contiguous(memory_format=torch.channels_last)
    blk = blk.to(memory_format=torch.channels_last)
    y = blk(x)  # fused (fp32 NHWC)
    blk_cpu = Bottleneck(64, 16)
    blk_cpu.load_state_dict({k: v.cpu() for k, v in blk.state_dict().items()})
    yr = blk_cpu(x.cpu())  # eager path
    torch.testing.assert_close(y.cpu(), yr, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("V,ld", [(50257, 50257), (50257, 50304), (1000, 1000), (130, 136)])
@pytest.mark.parametrize("shift", [False, True])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_fused_cross_entropy(cuda, V, ld, shift, dt):
    """K6 vs fp32 F.cross_entropy: loss and logit gradient, padded vocab, causal shift, ignore_index."""
    torch.manual_seed(9)
    B, S = 3, 17
    logits = (torch.randn(B, S, ld, device=cuda) * 3).to(dt).requires_grad_(True)
    tg = torch.randint(0, V, (B, S), device=cuda)
    tg[0, 3] = -100
    loss = ops.cross_entropy(logits, tg, shift=shift, vocab=V)
    loss.backward()
    lr = logits.detach().float().requires_grad_(True)
    l2, t2 = (lr[:, :-1], tg[:, 1:]) if shift else (lr, tg)
    ref = torch.nn.functional.cross_entropy(l2[..., :V].reshape(-1, V), t2.reshape(-1), ignore_index=-100)
    ref.backward()
    torch.testing.assert_close(loss.float(), ref, atol=2e-3, rtol=2e-3)
    tol = 2e-2 if dt == torch.bfloat16 else 1e-5
    torch.testing.assert_close(logits.grad.float(), lr.grad, atol=tol * lr.grad.abs().max().item() + 1e-7, rtol=tol)
    if ld > V:
        assert logits.grad[..., V:].abs().max() == 0


@pytest.mark.parametrize("fused", [True, False])
def test_cross_entropy_scale_is_folded_into_the_gradient(cuda, fused, monkeypatch):
    """``cross_entropy(..., scale=s)`` (a microbatched step's 1 / M, ops.scaled_loss) equals
    ``s * cross_entropy(...)`` in value and logit gradient, for the one-pass (K6f) and two-pass
    kernels -- and the one-pass gradient is finished at forward time (upstream gradient 1)."""
    monkeypatch.setattr(ops, "XENT_FUSED", fused)
    torch.manual_seed(4)
    V = 50257
    base = (torch.randn(2, 33, 50304, device=cuda) * 3).bfloat16()
    tg = torch.randint(0, V, (2, 33), device=cuda)
    a = base.clone().requires_grad_(True)
    la = ops.cross_entropy(a, tg, shift=True, vocab=V, scale=0.25)
    la.backward()
    b = base.clone().requires_grad_(True)
    lb = ops.cross_entropy(b, tg, shift=True, vocab=V)
    (lb * 0.25).backward()
    torch.testing.assert_close(la.float(), 0.25 * lb.detach().float(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(a.grad.float(), b.grad.float(), atol=1e-6, rtol=1e-2)


@pytest.mark.parametrize("V,ld", [(50257, 50304), (128256, 128256), (130, 136)])
def test_one_pass_cross_entropy_matches_two_pass(cuda, V, ld, monkeypatch):
    """K6f (loss + finished gradient in one pass over the logits, backward only rescales) against the
    two-pass K6 and fp32 F.cross_entropy, with an upstream gradient != 1 and ignored targets."""
    torch.manual_seed(5)
    B, S = 2, 9
    base = (torch.randn(B, S, ld, device=cuda) * 3).bfloat16()
    tg = torch.randint(0, V, (B, S), device=cuda)
    tg[1, 4] = -100
    assert ops._xent_fused_ok(base)
    grads, losses = [], []
    for fused in (True, False):
        monkeypatch.setattr(ops, "XENT_FUSED", fused)
        lg = base.clone().requires_grad_(True)
        loss = ops.cross_entropy(lg, tg, shift=True, vocab=V)
        (loss * 2.5).backward()
        grads.append(lg.grad.float())
        losses.append(loss.detach().float())
    lr = base.float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lr[:, :-1, :V].reshape(-1, V), tg[:, 1:].reshape(-1), ignore_index=-100)
    (ref * 2.5).backward()
    torch.testing.assert_close(losses[0], ref.detach(), atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(losses[0], losses[1], atol=1e-5, rtol=1e-5)
    scale = lr.grad.abs().max().item()
    torch.testing.assert_close(grads[0], lr.grad, atol=2e-2 * scale, rtol=2e-2)
    torch.testing.assert_close(grads[0], grads[1], atol=1e-2 * scale, rtol=1e-2)
    assert grads[0][:, :, V:].abs().sum() == 0 and grads[0][:, -1].abs().max() == 0
    assert grads[0][1, 3].abs().max() == 0  # the ignored target's row
    # the one-pass gradient is handed out once; a second backward says how to get two
    monkeypatch.setattr(ops, "XENT_FUSED", True)
    lg = base.clone().requires_grad_(True)
    loss = ops.cross_entropy(lg, tg, shift=True, vocab=V)
    loss.backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="MADNN_XENT_FUSED"):
        loss.backward()


@pytest.mark.parametrize("geom", [(3, 2, 1, 16, 16), (3, 2, 1, 15, 13), (2, 2, 0, 8, 10), (3, 1, 1, 9, 7),
                                  (5, 3, 2, 17, 11)])
@pytest.mark.parametrize("C", [8, 64, 200])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_maxpool_nhwc(cuda, geom, C, dt):
    """K7 NHWC max-pool fwd/bwd vs F.max_pool2d on the same (fp32-upcast) values: exact."""
    k, s, p, H, W = geom
    torch.manual_seed(11)
    x = torch.randn(3, C, H, W, device=cuda).to(dt).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    assert ops.max_pool_supported(x, k, s, p)
    y = ops.max_pool2d(x, k, s, p)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    yr = torch.nn.functional.max_pool2d(xr, k, s, p)
    yr.backward(dy.float())
    assert y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), yr, atol=0, rtol=0)
    tol = 1e-2 if dt == torch.bfloat16 else 1e-6  # overlapping windows sum in fp32, round once to bf16
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=tol, rtol=tol)
    with torch.no_grad():
        torch.testing.assert_close(ops.max_pool2d(x, k, s, p), y.detach(), atol=0, rtol=0)


def test_maxpool_module_fallback_and_resnet_stem(cuda):
    """FusedMaxPool2d: NCHW input falls back to ATen; the ResNet stem shape runs K7."""
    from madnn.nn import FusedMaxPool2d

    m = FusedMaxPool2d(3, 2, 1)
    x = torch.randn(2, 64, 112, 112, device=cuda).bfloat16()
    torch.testing.assert_close(m(x), torch.nn.functional.max_pool2d(x, 3, 2, 1))
    xc = x.contiguous(memory_format=torch.channels_last)
    assert ops.max_pool_supported(xc, 3, 2, 1)
    torch.testing.assert_close(m(xc), torch.nn.functional.max_pool2d(x, 3, 2, 1), atol=0, rtol=0)


@pytest.mark.parametrize("shape", [(4, 512, 1024), (3, 77, 4096), (1000, 264), (2, 64, 3072)])
@pytest.mark.parametrize("gelu", [False, True])
def test_bias_grad_k11(cuda, shape, gelu):
    """K11: column sum (and fused tanh-GELU backward) vs the fp32 PyTorch reference."""
    torch.manual_seed(5)
    dy = torch.randn(*shape, device=cuda).bfloat16()
    pre = torch.randn(*shape, device=cuda).bfloat16() * 2 if gelu else None
    db, dp = ops.bias_grad(dy, pre, torch.float32)
    g = dy.float()
    if gelu:
        pr = pre.float().requires_grad_(True)
        torch.nn.functional.gelu(pr, approximate="tanh").backward(g)
        g = pr.grad
        torch.testing.assert_close(dp.float(), g, atol=2e-2, rtol=1e-2)
    else:
        assert dp is None
    ref = g.reshape(-1, shape[-1]).sum(0)
    torch.testing.assert_close(db, ref, atol=1e-3 * ref.abs().max().item() + 1e-3, rtol=1e-3)


@pytest.mark.parametrize("gelu", [False, True])
def test_fused_linear_matches_eager(cuda, gelu):
    """ops.linear (K11 bias grad in the backward) == F.linear (+gelu) in output and all three grads."""
    torch.manual_seed(6)
    x = torch.randn(4, 128, 256, device=cuda).bfloat16().requires_grad_(True)
    w = (torch.randn(512, 256, device=cuda) * 0.05).bfloat16().requires_grad_(True)
    b = (torch.randn(512, device=cuda) * 0.1).bfloat16().requires_grad_(True)
    y = ops.linear(x, w, b, gelu=gelu)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.linear(xr, wr, br)
    if gelu:
        yr = torch.nn.functional.gelu(yr, approximate="tanh")
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    for a, r in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert a.dtype == torch.bfloat16
        torch.testing.assert_close(a.float(), r, atol=3e-2 * r.abs().max().item(), rtol=3e-2)


# ------------------------------------------------------- hipBLASLt epilogue Linear
@pytest.mark.parametrize("gelu,res,bias", [(True, False, True), (False, True, True), (True, True, False),
                                           (False, True, False)])
@pytest.mark.parametrize("M,K,N", [(512, 256, 1024), (333, 128, 64)])
def test_lt_linear_epilogues_match_fp32(cuda, gelu, res, bias, M, K, N):
    """One hipBLASLt GEMM with the bias / tanh-GELU (+ pre-activation AUX) / residual epilogue vs
    the fp32 composition; backward through ops.linear vs autograd of the fp32 reference."""
    torch.manual_seed(0)
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(N, K, device=cuda, dtype=torch.bfloat16) * K ** -0.5).requires_grad_()
    b = (torch.randn(N, device=cuda, dtype=torch.bfloat16) * 0.1).requires_grad_() if bias else None
    r = torch.randn(M, N, device=cuda, dtype=torch.bfloat16, requires_grad=True) if res else None
    # where hipBLASLt refuses this epilogue kind on the box (ops._LT_FAILED), ops.linear took its
    # fallback path: that path is what the comparisons below then verify, never skipped
    y = madnn.ops.linear(x, w, b, gelu=gelu, residual=r)
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    bf = b.detach().float().requires_grad_() if bias else None
    rf = r.detach().float().requires_grad_() if res else None
    yf = torch.nn.functional.linear(xf, wf, bf)
    yf = torch.nn.functional.gelu(yf, approximate="tanh") if gelu else yf
    yf = yf + rf if res else yf
    assert _rel(y, yf) < 1e-2
    g = torch.randn_like(yf)
    y.backward(g.to(y.dtype))
    yf.backward(g)
    assert _rel(x.grad, xf.grad) < 2e-2 and _rel(w.grad, wf.grad) < 2e-2
    if bias:
        assert _rel(b.grad, bf.grad) < 2e-2
    if res:
        assert _rel(r.grad, rf.grad) < 1e-2


def _rel(a, b):
    return float((a.detach().float() - b.detach().float()).norm() / b.detach().float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("choice", ["k12", "lt", "auto"])
@pytest.mark.parametrize("bias_dt", [torch.bfloat16, torch.float32, None])
def test_gelu_linear_forward_choices_match_fp32(cuda, monkeypatch, choice, bias_dt):
    """The GELU Linear forward through K12's fused bias + AUX + GELU epilogue, through hipBLASLt +
    the K11 GELU pass, and through the per-shape timed choice: output, saved pre-activation and
    all three gradients vs autograd of the fp32 composition."""
    monkeypatch.setattr(madnn.ops, "GELU_FWD", choice)
    monkeypatch.setitem(madnn.ops._LT_KIND, "gelu", False)  # hipBLASLt's GELU epilogue out of the way
    torch.manual_seed(11)
    M, K, N = 768, 320, 1032  # partial i / j tiles, K a multiple of 64
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(N, K, device=cuda, dtype=torch.bfloat16) * K ** -0.5).requires_grad_()
    b = (torch.randn(N, device=cuda, dtype=bias_dt) * 0.1).requires_grad_() if bias_dt else None
    y = madnn.ops.linear(x, w, b, gelu=True)
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    bf = b.detach().float().requires_grad_() if b is not None else None
    yf = torch.nn.functional.gelu(torch.nn.functional.linear(xf, wf, bf), approximate="tanh")
    assert y.dtype == torch.bfloat16 and _rel(y, yf) < 1e-2
    g = torch.randn_like(yf)
    y.backward(g.bfloat16())
    yf.backward(g)
    assert _rel(x.grad, xf.grad) < 2e-2 and _rel(w.grad, wf.grad) < 2e-2
    if b is not None:
        assert b.grad.dtype == bias_dt and _rel(b.grad, bf.grad) < 2e-2
    if choice == "auto":
        assert set(madnn.ops._GELU_FWD_CHOICE.values()) <= {"k12", "k12p", "lt"}


@pytest.mark.parametrize("rms", [False, True])
def test_norm_fork_gradient_joins_backward(cuda, rms):
    """fork=True: (N(x), x) where the alias's gradient is added inside the K3 backward pass."""
    torch.manual_seed(3)
    x = torch.randn(64, 1024, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.rand(1024, device=cuda) + 0.5).requires_grad_()
    b = None if rms else (torch.randn(1024, device=cuda) * 0.1).requires_grad_()
    fn = madnn.ops.rms_norm if rms else madnn.ops.layer_norm
    y, xa = fn(x, w, eps=1e-5, fork=True) if rms else fn(x, w, b, eps=1e-5, fork=True)
    g1, g2 = torch.randn_like(y), torch.randn_like(y)
    (y.float() * g1.float()).sum().add((xa.float() * g2.float()).sum()).backward()
    xr = x.detach().float().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    if rms:
        yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    else:
        yr = torch.nn.functional.layer_norm(xr, (1024,), wr, b.detach(), 1e-5)
    ((yr * g1.float()).sum() + (xr * g2.float()).sum()).backward()
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2


@pytest.mark.parametrize("shape,dt", [((4096, 4096), torch.bfloat16), ((333, 24), torch.float32),
                                      ((7, 8), torch.bfloat16)])
def test_gelu_fwd_kernel_matches_fp32(cuda, shape, dt):
    torch.manual_seed(4)
    x = (torch.randn(*shape, device=cuda) * 3).to(dt)
    x.view(-1)[:4] = torch.tensor([-30.0, 30.0, 0.0, -0.75], device=cuda).to(dt)  # saturation, zero, minimum
    y = madnn.ops.gelu_tanh(x)
    yr = torch.nn.functional.gelu(x.float(), approximate="tanh")
    assert y.dtype == dt
    torch.testing.assert_close(y.float(), yr, atol=1e-2 if dt == torch.bfloat16 else 1e-5,
                               rtol=1e-2 if dt == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("C", [64, 256, 2048])
@pytest.mark.parametrize("with_stats", [False, True])
def test_batchnorm_dual_residual_bn(cuda, C, with_stats):
    """K5 RAFF: relu(bn(x) + bn_r(r)) in one kernel pair vs fp32 eager: output, both BNs' running
    stats / nbt and every gradient (x, r, both weights and biases)."""
    from madnn.nn.norm import FusedBatchNorm2d

    torch.manual_seed(9)
    N, H, W = 6, 7, 9
    x = (torch.randn(N, C, H, W, device=cuda) * 1.5 + 0.3).bfloat16().contiguous(memory_format=torch.channels_last)
    r = (torch.randn(N, C, H, W, device=cuda) * 0.7 - 0.2).bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    r.requires_grad_(True)
    bn, bn_r = FusedBatchNorm2d(C).to(cuda), FusedBatchNorm2d(C).to(cuda)
    with torch.no_grad():
        for m in (bn, bn_r):
            m.weight.uniform_(0.5, 1.5)
            m.bias.normal_(0, 0.1)
    ref_bn, ref_bn_r = torch.nn.BatchNorm2d(C).to(cuda), torch.nn.BatchNorm2d(C).to(cuda)
    ref_bn.load_state_dict(bn.state_dict())
    ref_bn_r.load_state_dict(bn_r.state_dict())
    st = st_r = None
    if with_stats:  # producer-epilogue format: [rows, 2, C] partial (sum, sum of squares)
        def part(t):
            v = t.detach().float().permute(0, 2, 3, 1).reshape(3, -1, C)
            return torch.stack([v.sum(1), (v * v).sum(1)], 1).contiguous()
        st, st_r = part(x), part(r)
    assert ops.batch_norm_dual_supported(x, r, bn, bn_r)
    y = ops.batch_norm_add_bn_relu(x, r, bn, bn_r, st, st_r)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True)
    yr = torch.relu(ref_bn(xr) + ref_bn_r(rr))
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    for m, mr in ((bn, ref_bn), (bn_r, ref_bn_r)):
        torch.testing.assert_close(m.running_mean, mr.running_mean, atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(m.running_var, mr.running_var, atol=1e-3, rtol=1e-3)
        assert int(m.num_batches_tracked) == 1
        torch.testing.assert_close(m.weight.grad, mr.weight.grad, atol=0.15, rtol=0.05)
        torch.testing.assert_close(m.bias.grad, mr.bias.grad, atol=0.15, rtol=0.05)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=9e-2, rtol=9e-2)
    torch.testing.assert_close(r.grad.float(), rr.grad, atol=9e-2, rtol=9e-2)


def test_resnet50_downsample_block_dual_bn_matches_composition(cuda):
    """A downsample Bottleneck with the dual BN path vs the same block with it switched off."""
    import madnn.models.resnet as R

    torch.manual_seed(10)
    ds = torch.nn.Sequential(R.conv1x1(64, 256, 2), R.BN(256))
    blk = R.Bottleneck(64, 64, 2, ds).to(cuda).bfloat16()
    for m in blk.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.float()
            torch.nn.init.uniform_(m.weight, 0.5, 1.5)
    import copy
    blk2 = copy.deepcopy(blk)
    assert blk._dual_bn()
    x = torch.randn(8, 64, 28, 28, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    y1 = blk(x1)
    old = R._DUAL_BN
    R._DUAL_BN = False
    try:
        assert not blk2._dual_bn()
        y2 = blk2(x2)
    finally:
        R._DUAL_BN = old
    # fp32 copy of the same block (eager convolutions, composed BNs) as the oracle: bf16 ReLU-mask
    # flips make two bf16 paths differ element-wise, so compare each path's error against fp32
    blk3 = copy.deepcopy(blk2).float()
    x3 = x.float().requires_grad_(True)
    y3 = blk3(x3)
    dy = torch.randn_like(y1)
    y1.backward(dy)
    y2.backward(dy)
    y3.backward(dy.float())

    def rel(a, b):
        return ((a.float() - b).norm() / b.norm()).item()

    assert rel(y1, y3) <= 1.5 * rel(y2, y3) + 1e-3
    assert rel(x1.grad, x3.grad) <= 1.5 * rel(x2.grad, x3.grad) + 1e-3
    assert rel(x1.grad, x3.grad) < 0.1   # bf16 end to end through a whole block: ~0.06
    for (n, p1), p2, p3 in zip(blk.named_parameters(), blk2.parameters(), blk3.parameters()):
        assert rel(p1.grad, p3.grad) <= 1.5 * rel(p2.grad, p3.grad) + 2e-3, n
    for (n, b1), b2 in zip(blk.named_buffers(), blk2.buffers()):
        torch.testing.assert_close(b1.float(), b2.float(), atol=1e-3, rtol=1e-3, msg=n)


@pytest.mark.parametrize("shape", [(4, 64, 112, 112), (3, 64, 17, 23), (2, 128, 9, 8), (2, 8, 6, 5)])
@pytest.mark.parametrize("with_stats", [False, True])
def test_bn_relu_maxpool_fused_matches_fp32(cuda, shape, with_stats):
    """K7+K5 stem fusion: maxpool3x3/s2(relu(bn(y))) with the BN apply in the pool's loads and the
    pool gradient gathered inside the BN backward vs fp32 eager: output, running stats, all grads."""
    from madnn.nn.norm import FusedBatchNorm2d, FusedMaxPool2d

    n, c, h, w = shape
    torch.manual_seed(11)
    y = (torch.randn(n, c, h, w, device=cuda) * 1.2 + 0.1).bfloat16().contiguous(memory_format=torch.channels_last)
    y.requires_grad_(True)
    bn = FusedBatchNorm2d(c).to(cuda)
    with torch.no_grad():
        bn.weight.uniform_(-0.5, 1.5)   # negative scales too: max of the affine is not the affine of the max
        bn.bias.normal_(0, 0.3)
    pool = FusedMaxPool2d(3, 2, 1)
    ref = torch.nn.BatchNorm2d(c).to(cuda)
    ref.load_state_dict(bn.state_dict())
    st = None
    if with_stats:
        v = y.detach().float().permute(0, 2, 3, 1).reshape(1, -1, c)
        st = torch.stack([v.sum(1), (v * v).sum(1)], 1).contiguous()
    assert ops.bn_relu_maxpool_supported(y, bn, pool)
    out = ops.bn_relu_maxpool(y, bn, pool, st)
    dp = torch.randn_like(out)
    out.backward(dp)
    yr = y.detach().float().requires_grad_(True)
    outr = torch.nn.functional.max_pool2d(torch.relu(ref(yr)), 3, 2, 1)
    outr.backward(dp.float())
    torch.testing.assert_close(out.float(), outr, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(bn.running_var, ref.running_var, atol=1e-3, rtol=1e-3)
    assert int(bn.num_batches_tracked) == 1
    # bf16 rounding of relu(bn(y)) can move an argmax between near-equal window values, so the
    # input gradient is compared in norm; the parameter gradients (sums) element-wise
    rel = ((y.grad.float() - yr.grad).norm() / yr.grad.norm()).item()
    assert rel < 0.05, rel
    torch.testing.assert_close(bn.weight.grad, ref.weight.grad, atol=0.2, rtol=0.05)
    torch.testing.assert_close(bn.bias.grad, ref.bias.grad, atol=0.2, rtol=0.05)


def test_batchnorm_apply_walk_variants_bitwise(cuda):
    """The BN apply walks with and without coefficient hoisting (the per-chunk reload is also the
    path for grid strides that are not a multiple of C) are pure scheduling changes: outputs and
    gradients must be bitwise identical."""
    import ctypes

    from madnn.nn.norm import FusedBatchNorm2d

    tune = ctypes.CDLL(str(ops.kernels_path())).madnn_bn_tune
    torch.manual_seed(12)
    C = 256
    x = torch.randn(16, C, 56, 56, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x)
    dy = torch.randn_like(x)
    bn, bn_r = FusedBatchNorm2d(C).to(cuda), FusedBatchNorm2d(C).to(cuda)
    outs = []
    old = tune(2, -1)
    assert tune(3, -1) == -1   # the multi-chunk walks are gone
    try:
        for hoist in (0, 1):
            tune(2, hoist)
            res = []
            for dual in (False, True):
                xa, ra = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
                y = ops.batch_norm_add_bn_relu(xa, ra, bn, bn_r) if dual else \
                    ops.batch_norm_act(xa, bn.weight, bn.bias, None, None, training=True, relu=True, residual=ra)
                y.backward(dy)
                res += [y.detach(), xa.grad, ra.grad]
            outs.append(res)
    finally:
        tune(2, old)
    for k, (a, b) in enumerate(zip(outs[0], outs[1])):
        assert torch.equal(a, b), k


def test_batchnorm_many_producer_partial_rows(cuda):
    """Producer statistics with thousands of partial rows (K13's one row per 256-pixel tile) are
    folded before the finalize: running stats and outputs equal the statistics-pass path."""
    torch.manual_seed(13)
    C = 64
    x = (torch.randn(8, C, 64, 96, device=cuda) * 2 + 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
    v = x.float().permute(0, 2, 3, 1).reshape(-1, C)
    rows = torch.arange(v.size(0), device=cuda) % 3001   # 3001 uneven row groups
    part = torch.zeros(3001, 2, C, device=cuda)
    part[:, 0].index_add_(0, rows, v)
    part[:, 1].index_add_(0, rows, v * v)
    w, b = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda)
    rm1, rv1 = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    rm2, rv2 = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y1 = ops.batch_norm_act(x, w, b, rm1, rv1, training=True, relu=True)
    y2 = ops.batch_norm_act(x, w, b, rm2, rv2, training=True, relu=True, stats=part)
    torch.testing.assert_close(rm1, rm2, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rv1, rv2, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(y1.float(), y2.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("mode", ["plain", "fork", "residual"])
def test_norm_colsum_feeds_linear_bias_grad(cuda, monkeypatch, mode):
    """A biased Linear feeding a K3 norm: the norm backward's dx column sums become the Linear's bias
    gradient (no separate column-sum pass) -- equal to the fp32 reference in every norm mode."""
    calls = []
    real = madnn.ops.bias_grad
    monkeypatch.setattr(madnn.ops, "bias_grad", lambda *a, **k: calls.append(1) or real(*a, **k))
    torch.manual_seed(12)
    x = torch.randn(4, 96, 256, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(512, 256, device=cuda, dtype=torch.bfloat16) * 0.06).requires_grad_()
    b = (torch.randn(512, device=cuda, dtype=torch.bfloat16) * 0.1).requires_grad_()
    lw = (torch.rand(512, device=cuda) + 0.5).requires_grad_()
    lb = (torch.randn(512, device=cuda) * 0.1).requires_grad_()
    r = torch.randn(4, 96, 512, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    g1, g2 = torch.randn(4, 96, 512, device=cuda), torch.randn(4, 96, 512, device=cuda)

    def run(xx, ww, bb, rr, lin, norm):
        h = lin(xx, ww, bb)
        if mode == "plain":
            return (norm(h, None).float() * g1).sum()
        if mode == "fork":
            y, ha = norm(h, "fork")
            return (y.float() * g1).sum() + (ha.float() * g2).sum()
        y, s = norm(h, rr)
        return (y.float() * g1).sum() + (s.float() * g2).sum()

    def mnorm(h, arg):
        if arg == "fork":
            return madnn.ops.layer_norm(h, lw, lb, fork=True)
        if arg is None:
            return madnn.ops.layer_norm(h, lw, lb)
        return madnn.ops.layer_norm(h, lw, lb, residual=arg)

    run(x, w, b, r, lambda a, ww, bb: madnn.ops.linear(a, ww, bb), mnorm).backward()
    assert not calls, "the Linear ran its own bias column-sum pass"
    xf, wf, bf, rf = (t.detach().float().requires_grad_() for t in (x, w, b, r))
    lwf, lbf = lw.detach().clone().requires_grad_(), lb.detach().clone().requires_grad_()

    def fnorm(h, arg):
        if arg == "fork":
            return torch.nn.functional.layer_norm(h, (512,), lwf, lbf), h
        if arg is None:
            return torch.nn.functional.layer_norm(h, (512,), lwf, lbf)
        s = h + arg
        return torch.nn.functional.layer_norm(s, (512,), lwf, lbf), s

    run(xf, wf, bf, rf, torch.nn.functional.linear, fnorm).backward()
    assert _rel(b.grad, bf.grad) < 2e-2 and _rel(w.grad, wf.grad) < 2e-2 and _rel(x.grad, xf.grad) < 2e-2


@pytest.mark.parametrize("second", ["add", "inplace"])
def test_linear_bias_grad_with_two_consumers(cuda, second):
    """A biased Linear whose output feeds the LayerNorm (which hands the Linear its bias gradient
    as a column sum of the gradient it produces) AND another op: the accumulated gradient is no
    longer the one the column sum describes, so the bias gradient must come from the sum (ADVICE
    r3: version-stamped side channels)."""
    torch.manual_seed(0)
    M, K, N = 256, 128, 256
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(N, K, device=cuda, dtype=torch.bfloat16) * K ** -0.5).requires_grad_()
    b = (torch.randn(N, device=cuda, dtype=torch.bfloat16) * 0.1).requires_grad_()
    lw = torch.ones(N, device=cuda, dtype=torch.float32, requires_grad=True)
    lb = torch.zeros(N, device=cuda, dtype=torch.float32, requires_grad=True)

    def fwd(xx, ww, bb, lww, lbb, ref):
        y = madnn.ops.linear(xx, ww, bb) if not ref else torch.nn.functional.linear(xx, ww, bb)
        z = madnn.ops.layer_norm(y, lww, lbb) if not ref else torch.nn.functional.layer_norm(y, (N,), lww, lbb)
        if second == "add":
            return z.float().sum() + (y.float() * 3.0).sum()
        y2 = y * 1.0
        y2.mul_(3.0)
        return z.float().sum() + y2.float().sum()

    fwd(x, w, b, lw, lb, False).backward()
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
    lwf, lbf = lw.detach().clone().requires_grad_(), lb.detach().clone().requires_grad_()
    fwd(xf, wf, bf, lwf, lbf, True).backward()
    assert _rel(b.grad, bf.grad) < 2e-2
    assert _rel(w.grad, wf.grad) < 3e-2


@pytest.mark.parametrize("V,ld", [(50257, 50304), (130, 136), (1000, 1000)])
def test_one_pass_cross_entropy_ragged_vocab(cuda, V, ld, monkeypatch):
    """The fused one-pass kernel (v_exp_f32 on whole chunks, per-element vocabulary-end test on the
    straddling chunk) on padded and unpadded vocabularies vs fp32 F.cross_entropy."""
    monkeypatch.setattr(ops, "XENT_FUSED", True)
    torch.manual_seed(8)
    B, S = 2, 9
    base = (torch.randn(B, S, ld, device=cuda) * 3).bfloat16()
    tg = torch.randint(0, V, (B, S), device=cuda)
    tg[0, 2] = -100
    lg = base.clone().requires_grad_(True)
    loss = ops.cross_entropy(lg, tg, shift=True, vocab=V)
    loss.backward()
    lr = base.float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lr[:, :-1, :V].reshape(-1, V), tg[:, 1:].reshape(-1), ignore_index=-100)
    ref.backward()
    torch.testing.assert_close(loss.float(), ref, atol=2e-3, rtol=2e-3)
    g = lg.grad.float()
    torch.testing.assert_close(g, lr.grad, atol=2e-2 * lr.grad.abs().max().item() + 1e-7, rtol=2e-2)
    if ld > V:
        assert lg.grad[..., V:].abs().max() == 0
