"""K12P persistent GEMM (madnn/ops/csrc/gemmp.hip) against plain PyTorch fp32 references.

Shapes: one tile, fewer tiles than 8 (fewer XCD labels than XCDs), uneven tile ranges per XCD
label, and more tiles than CUs (several tiles per workgroup: the DMA stream and the counted waits
run across epilogues).  Variants: plain, fp32 / bf16 bias, bias + tanh-GELU with the
pre-activation stored, data gradient plain and with the dGELU epilogue + fused column sums.
The GELU epilogues must equal the unfused K11 passes bitwise (same formula, same roundings)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ops():
    from madnn import ops

    assert ops.load_kernels(), "HIP kernel library failed to load"
    return torch.ops.madnn


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


# (M tokens, N out features, K reduction)
SHAPES = [(256, 256, 64), (512, 768, 128), (256 * 37, 768, 256), (16384, 2048, 512), (8192, 4096, 1024)]


def _data(M, N, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * K ** -0.5).bfloat16()
    return g, x, w


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_linear_fwd_p_plain_and_bias(cuda, M, N, K):
    m = _ops()
    g, x, w = _data(M, N, K, M + N + K)
    assert m.gemmp_supported(N, M, K, True)
    y, aux = m.linear_fwd_p(x, w, None, 0)
    ref = x.float() @ w.float().t()
    assert y.shape == (M, N) and aux.numel() == 0
    assert _rel(y, ref) < 5e-3
    # same accumulation as the one-tile-per-workgroup K12: bitwise equal
    y12, _ = m.linear_fwd(x, w, None, None, 0, False)
    assert torch.equal(y, y12)
    for bdt in (torch.float32, torch.bfloat16):
        b = torch.randn(N, device="cuda", generator=g).to(bdt)
        yb, _ = m.linear_fwd_p(x, w, b, 0)
        torch.testing.assert_close(yb.float(), ref + b.float(), atol=3e-2, rtol=2e-2)
        yb12, _ = m.linear_fwd(x, w, b, None, 0, False)
        assert torch.equal(yb, yb12)


@pytest.mark.parametrize("kind,approx", [(1, "tanh"), (2, "none")])
@pytest.mark.parametrize("M,N,K", SHAPES[1:])
def test_linear_fwd_p_gelu_epilogue(cuda, M, N, K, kind, approx):
    m = _ops()
    g, x, w = _data(M, N, K, 3 * M + N)
    b = torch.randn(N, device="cuda", generator=g) * 0.5
    y, pre = m.linear_fwd_p(x, w, b, kind)
    ref_pre = x.float() @ w.float().t() + b
    torch.testing.assert_close(pre.float(), ref_pre, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(y.float(), F.gelu(ref_pre, approximate=approx), atol=3e-2, rtol=2e-2)
    # the fused epilogue rounds exactly as the standalone K11 GELU pass over the same pre-activation
    assert torch.equal(y, m.gelu_fwd(pre, kind))
    # and K11 matches F.gelu on the same bf16 input to the output rounding
    torch.testing.assert_close(y.float(), F.gelu(pre.float(), approximate=approx), atol=1e-2, rtol=8e-3)


# data gradient of a Linear(K -> N): dx[M, K] = dy[M, N] w[N, K] (K12P's output features = K)
DSHAPES = [(256, 64, 256), (512, 128, 768), (256 * 37, 256, 768), (16384, 512, 2048), (8192, 1024, 4096)]


def _ddata(M, N, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    dy = (torch.rand(M, N, device="cuda", generator=g) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * N ** -0.5).bfloat16()
    return g, dy, w


@pytest.mark.parametrize("M,N,K", DSHAPES)
def test_linear_dgrad_p_plain(cuda, M, N, K):
    m = _ops()
    g, dy, w = _ddata(M, N, K, 5 * M + K)
    dx, db = m.linear_dgrad_p(dy, w, None, torch.float32)
    ref = dy.float() @ w.float()
    assert dx.shape == (M, K) and db.numel() == 0
    assert _rel(dx, ref) < 5e-3
    assert torch.equal(dx, m.linear_dgrad(dy, w, None, False))


@pytest.mark.parametrize("kind,approx", [(1, "tanh"), (2, "none")])
@pytest.mark.parametrize("M,N,K", DSHAPES[1:])
@pytest.mark.parametrize("bias_dtype", [torch.float32, torch.bfloat16])
def test_linear_dgrad_p_dgelu_colsum(cuda, M, N, K, bias_dtype, kind, approx):
    """c_proj's data gradient with c_fc's GELU backward and bias gradient fused: against the fp32
    reference and bitwise against the unfused path (K12 dgrad, then the K11 dGELU + bias pass)."""
    m = _ops()
    g, dy, w = _ddata(M, N, K, 7 * M + N)
    pre = (torch.randn(M, K, device="cuda", generator=g) * 2).bfloat16()
    dh, db = m.linear_dgrad_p(dy, w, pre, bias_dtype, kind)
    da = (dy.float() @ w.float()).bfloat16().float()
    pf = pre.float().requires_grad_(True)
    F.gelu(pf, approximate=approx).backward(da)
    ref = pf.grad
    torch.testing.assert_close(dh.float(), ref, atol=4e-2, rtol=3e-2)
    assert db.dtype == bias_dtype and db.shape == (K,)
    torch.testing.assert_close(db.float(), ref.sum(0), atol=2e-1 + 2e-3 * M ** 0.5, rtol=2e-2)
    # unfused: the K12 data gradient, then the K11 dGELU + column-sum pass
    da12 = m.linear_dgrad(dy, w, None, False)
    db11, dh11 = m.bias_grad(da12, pre, bias_dtype, kind)
    assert torch.equal(dh, dh11)
    # same fp32 sums in another order; a bf16 bias gradient may then round one ulp apart
    tol = 1e-4 if bias_dtype == torch.float32 else 8e-3
    torch.testing.assert_close(db.float(), db11.float(), atol=1e-3 * M ** 0.5, rtol=tol)


def test_gemmp_refuses_edge_tiles(cuda):
    m = _ops()
    assert not m.gemmp_supported(300, 256, 64, False)    # ragged output features
    assert not m.gemmp_supported(256, 300, 64, False)    # ragged tokens
    assert not m.gemmp_supported(256, 256, 96, False)    # reduction not a multiple of 64
    assert not m.gemmp_supported(16384, 256, 64, True)   # bias larger than its LDS slot
    x = torch.zeros(300, 64, device="cuda", dtype=torch.bfloat16)
    w = torch.zeros(256, 64, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        m.linear_fwd_p(x, w, None, 0)


@pytest.mark.parametrize("approx", ["tanh", "none"])
@pytest.mark.parametrize("impl", ["k12p", "lt"])
def test_gelu_mlp_node_against_fp32(cuda, impl, approx, monkeypatch):
    """GPT-2's MLP as one autograd node (ops.gelu_mlp) with the K12P epilogues forced, and with the
    hipBLASLt + K11 path forced: forward and every gradient against fp32 eager autograd."""
    from madnn import ops

    monkeypatch.setattr(ops, "GELU_FWD", impl)
    monkeypatch.setattr(ops, "DGELU", impl)
    torch.manual_seed(0)
    B, S, H = 2, 512, 256
    x = torch.randn(B, S, H, device="cuda").bfloat16().requires_grad_(True)
    r = torch.randn(B, S, H, device="cuda").bfloat16().requires_grad_(True)
    w1 = (torch.randn(4 * H, H, device="cuda") * H ** -0.5).bfloat16().requires_grad_(True)
    b1 = (torch.randn(4 * H, device="cuda") * 0.1).requires_grad_(True)
    w2 = (torch.randn(H, 4 * H, device="cuda") * (4 * H) ** -0.5).bfloat16().requires_grad_(True)
    b2 = (torch.randn(H, device="cuda") * 0.1).requires_grad_(True)
    y = ops.gelu_mlp(x, w1, b1, w2, b2, r, approximate=approx)
    gy = torch.randn_like(y)
    got = torch.autograd.grad(y, (x, w1, b1, w2, b2, r), gy)
    xs = [t.detach().float().requires_grad_(True) for t in (x, w1, b1, w2, b2, r)]
    ref_y = F.linear(F.gelu(F.linear(xs[0], xs[1], xs[2]), approximate=approx), xs[3], xs[4]) + xs[5]
    ref = torch.autograd.grad(ref_y, xs, gy.float())
    assert _rel(y, ref_y) < 1e-2
    for name, a, b in zip(("dx", "dw1", "db1", "dw2", "db2", "dres"), got, ref):
        assert a.dtype == b.dtype or a.dtype == torch.bfloat16, name
        assert _rel(a, b) < 2e-2, (name, _rel(a, b))


@pytest.mark.parametrize("impl", ["k12", "lt"])
def test_gelu_mlp_erf_on_ragged_rows(cuda, impl, monkeypatch):
    """Rows that are not a multiple of 256 (no K12P): the exact-GELU MLP on K12's one-tile epilogue
    (or hipBLASLt + K11) and the K11 erf dGELU pass, against fp32 eager autograd."""
    from madnn import ops

    monkeypatch.setattr(ops, "GELU_FWD", impl)
    torch.manual_seed(3)
    x = torch.randn(300, 256, device="cuda").bfloat16().requires_grad_(True)
    w1 = (torch.randn(1024, 256, device="cuda") * 256 ** -0.5).bfloat16().requires_grad_(True)
    b1 = (torch.randn(1024, device="cuda") * 0.1).requires_grad_(True)
    w2 = (torch.randn(256, 1024, device="cuda") * 1024 ** -0.5).bfloat16().requires_grad_(True)
    b2 = (torch.randn(256, device="cuda") * 0.1).requires_grad_(True)
    y = ops.gelu_mlp(x, w1, b1, w2, b2, approximate="none")
    gy = torch.randn_like(y)
    got = torch.autograd.grad(y, (x, w1, b1, w2, b2), gy)
    xs = [t.detach().float().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    ref_y = F.linear(F.gelu(F.linear(xs[0], xs[1], xs[2])), xs[3], xs[4])
    ref = torch.autograd.grad(ref_y, xs, gy.float())
    assert _rel(y, ref_y) < 1e-2
    for name, a, b in zip(("dx", "dw1", "db1", "dw2", "db2"), got, ref):
        assert _rel(a, b) < 2e-2, (name, _rel(a, b))


def test_gelu_mlp_residual_is_input(cuda):
    """A post-LN block's ``y + MLP(y)``: the residual is the MLP's own input; its gradient is added
    inside the input's data-gradient GEMM (beta = 1) -- equal to fp32 eager autograd."""
    from madnn import ops

    torch.manual_seed(4)
    x = torch.randn(2, 512, 256, device="cuda").bfloat16().requires_grad_(True)
    w1 = (torch.randn(1024, 256, device="cuda") * 256 ** -0.5).bfloat16().requires_grad_(True)
    b1 = (torch.randn(1024, device="cuda") * 0.1).requires_grad_(True)
    w2 = (torch.randn(256, 1024, device="cuda") * 1024 ** -0.5).bfloat16().requires_grad_(True)
    b2 = (torch.randn(256, device="cuda") * 0.1).requires_grad_(True)
    y = ops.gelu_mlp(x, w1, b1, w2, b2, residual=x, approximate="none")
    gy = torch.randn_like(y)
    got = torch.autograd.grad(y, (x, w1, b1, w2, b2), gy)
    xs = [t.detach().float().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    ref_y = F.linear(F.gelu(F.linear(xs[0], xs[1], xs[2])), xs[3], xs[4]) + xs[0]
    ref = torch.autograd.grad(ref_y, xs, gy.float())
    assert _rel(y, ref_y) < 1e-2
    for name, a, b in zip(("dx", "dw1", "db1", "dw2", "db2"), got, ref):
        assert _rel(a, b) < 2e-2, (name, _rel(a, b))


def test_bert_layer_residual_tee_matches_eager(cuda, monkeypatch):
    """BERT's post-LN sublayers with both residual gradients folded into data-gradient GEMMs (attention:
    ops.linear_tee on the QKV projection; MLP: gelu_mlp(residual=y)) vs the same model with the fused
    Linear paths off: loss and every gradient agree (bf16)."""
    from madnn import ops
    from madnn.models.bert import BertForPreTraining, bert_config

    torch.manual_seed(3)
    cfg = bert_config("bert-tiny", hidden=256, heads=4, intermediate=512, layers=2)
    model = BertForPreTraining(cfg).to(cuda).bfloat16()
    ids = torch.randint(0, cfg.vocab_size, (2, 128), device=cuda)
    calls = []
    real = ops._LinearTeeFn.apply
    monkeypatch.setattr(ops._LinearTeeFn, "apply", lambda *a: calls.append(1) or real(*a))
    loss = model.loss_fn(model(ids), ids)
    loss.backward()
    assert len(calls) == cfg.layers
    got = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    model.zero_grad()
    monkeypatch.setattr(ops, "FUSED_LINEAR", False)
    loss2 = model.loss_fn(model(ids), ids)
    loss2.backward()
    torch.testing.assert_close(loss.float(), loss2.float(), atol=2e-2, rtol=2e-2)
    for n, p in model.named_parameters():
        assert _rel(got[n], p.grad) < 5e-2, (n, _rel(got[n], p.grad))


@pytest.mark.parametrize("M,O,I", [(4096, 3072, 1024), (1000, 1024, 4096)])
def test_dgrad_plus_kn_weight_gemm_matches_fp32(cuda, M, O, I):
    """ops._dgrad_plus: g @ W + r as one hipBLASLt GEMM reading W [O, I] untransposed (op N) with r as
    the C operand, vs fp32."""
    from madnn import ops

    torch.manual_seed(5)
    g = torch.randn(M, O, device=cuda).bfloat16()
    w = (torch.randn(O, I, device=cuda) * O ** -0.5).bfloat16()
    r = torch.randn(M, I, device=cuda).bfloat16()
    out = ops._dgrad_plus(g, w, r)
    assert not ops._LT_KN_FAILED, ops._LT_KN_FAILED
    ref = g.float() @ w.float() + r.float()
    assert out.dtype == torch.bfloat16 and out.shape == (M, I)
    assert _rel(out, ref) < 1e-2
