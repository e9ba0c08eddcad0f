"""K8 MFMA flash attention vs an fp32 SDPA reference on the same bf16 inputs.

Covers head dims 64/128, causal and full, grouped-query heads, sequence lengths that are not
multiples of the 64/128 tiles, strided (packed-QKV) inputs and the in-place dQKV path."""
import pytest
import torch
import torch.nn.functional as F

from madnn import ops

pytestmark = pytest.mark.gpu


def _ref(q, k, v, causal, scale):
    h, hkv = q.size(2), k.size(2)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=causal,
                                       scale=scale, enable_gqa=h != hkv)
    return o.transpose(1, 2)


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


CASES = [
    (2, 256, 4, 4, 64, True),
    (2, 256, 4, 4, 64, False),
    (1, 200, 4, 2, 64, True),
    (1, 77, 3, 3, 64, False),
    (2, 384, 4, 1, 128, True),
    (1, 130, 2, 2, 128, False),
    (1, 200, 4, 2, 128, True),    # D = 128 dQ key-half split on a ragged causal edge
    (1, 1024, 16, 16, 64, True),
]


@pytest.mark.parametrize("B,S,H,HKV,D,causal", CASES)
def test_attention_fwd_bwd(cuda, B, S, H, HKV, D, causal):
    torch.manual_seed(0)
    q = torch.randn(B, S, H, D, device=cuda).bfloat16().requires_grad_(True)
    k = torch.randn(B, S, HKV, D, device=cuda).bfloat16().requires_grad_(True)
    v = torch.randn(B, S, HKV, D, device=cuda).bfloat16().requires_grad_(True)
    scale = D ** -0.5
    o = ops.attention(q, k, v, causal=causal)
    assert o.shape == (B, S, H, D) and o.is_contiguous()
    do = torch.randn_like(o)
    o.backward(do)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = _ref(qr, kr, vr, causal, scale)
    orf.backward(do.float())
    assert _rel(o, orf) < 1e-2
    torch.testing.assert_close(o.float(), orf, atol=3e-2, rtol=3e-2)
    for g, gr, name in ((q.grad, qr.grad, "dq"), (k.grad, kr.grad, "dk"), (v.grad, vr.grad, "dv")):
        assert _rel(g, gr) < 2e-2, name


@pytest.mark.parametrize("B,S,H,HKV,D", [(1, 4096, 32, 8, 128), (2, 2048, 16, 16, 64)])
def test_attention_bench_shapes_causal(cuda, B, S, H, HKV, D):
    """The shapes the benches time: Llama-3 8B's (S = 4096, D = 128, GQA 32 / 8) and a long
    D = 64 case, causal, forward and all three gradients against fp32 SDPA (the reference runs
    one query-head group at a time to bound its memory)."""
    torch.manual_seed(4)
    q = torch.randn(B, S, H, D, device=cuda).bfloat16().requires_grad_(True)
    k = torch.randn(B, S, HKV, D, device=cuda).bfloat16().requires_grad_(True)
    v = torch.randn(B, S, HKV, D, device=cuda).bfloat16().requires_grad_(True)
    o = ops.attention(q, k, v, causal=True)
    do = torch.randn_like(o)
    gq, gk, gv = torch.autograd.grad(o, (q, k, v), do)
    g = H // HKV
    rq, rk, rv = torch.zeros_like(gq, dtype=torch.float32), torch.zeros_like(gk, dtype=torch.float32), \
        torch.zeros_like(gv, dtype=torch.float32)
    orf = torch.empty_like(o, dtype=torch.float32)
    for j in range(HKV):   # kv head j and its g query heads
        qs = slice(j * g, (j + 1) * g)
        qr = q[:, :, qs].detach().float().requires_grad_(True)
        kr = k[:, :, j:j + 1].detach().float().requires_grad_(True)
        vr = v[:, :, j:j + 1].detach().float().requires_grad_(True)
        oj = _ref(qr, kr, vr, True, D ** -0.5)
        a, b, c = torch.autograd.grad(oj, (qr, kr, vr), do[:, :, qs].float())
        orf[:, :, qs], rq[:, :, qs], rk[:, :, j:j + 1], rv[:, :, j:j + 1] = oj.detach(), a, b, c
    assert _rel(o, orf) < 1e-2, _rel(o, orf)
    for got, ref, name in ((gq, rq, "dq"), (gk, rk, "dk"), (gv, rv, "dv")):
        assert _rel(got, ref) < 2e-2, (name, _rel(got, ref))


@pytest.mark.parametrize("H,HKV,D", [(4, 4, 64), (8, 2, 128)])
def test_attention_qkvpacked_inplace_grad(cuda, H, HKV, D):
    torch.manual_seed(1)
    B, S = 2, 192
    qkv = torch.randn(B, S, H + 2 * HKV, D, device=cuda).bfloat16().requires_grad_(True)
    o = ops.attention_qkvpacked(qkv, H, HKV, causal=True)
    do = torch.randn_like(o)
    o.backward(do)
    ref = qkv.detach().float().requires_grad_(True)
    q, k, v = ref.split([H, HKV, HKV], dim=2)
    orf = _ref(q, k, v, True, D ** -0.5)
    orf.backward(do.float())
    assert _rel(o, orf) < 1e-2
    assert _rel(qkv.grad, ref.grad) < 2e-2


def test_attention_edge_rows_exact_softmax(cuda):
    """A query that sees exactly one key (causal row 0) returns that value row; fully masked padding
    rows of the last tile do not leak into valid rows."""
    torch.manual_seed(2)
    q = torch.randn(1, 65, 1, 64, device=cuda).bfloat16()
    k = torch.randn(1, 65, 1, 64, device=cuda).bfloat16()
    v = torch.randn(1, 65, 1, 64, device=cuda).bfloat16()
    o = ops.attention(q, k, v, causal=True)
    torch.testing.assert_close(o[0, 0, 0].float(), v[0, 0, 0].float(), atol=1e-2, rtol=0)


def test_selfattention_module_uses_k8_and_matches_sdpa(cuda):
    from madnn.models.common import RotaryEmbedding, SelfAttention

    torch.manual_seed(3)
    for rope in (None, RotaryEmbedding(64)):
        m = SelfAttention(256, 4, kv_heads=2 if rope is not None else None, rope=rope).to(cuda).bfloat16()
        x = torch.randn(2, 96, 256, device=cuda).bfloat16().requires_grad_(True)
        y = m(x)
        y.float().square().mean().backward()
        gx = x.grad.clone()
        x.grad = None
        m.zero_grad()
        orig = ops.attention_supported
        try:
            ops.attention_supported = lambda *a, **k: False
            y2 = m(x)
            y2.float().square().mean().backward()
        finally:
            ops.attention_supported = orig
        assert _rel(y, y2) < 1e-2
        assert _rel(gx, x.grad) < 3e-2


@pytest.mark.parametrize("H,HKV,D,S", [(4, 4, 64, 256), (8, 2, 128, 200)])
def test_qkv_bias_grad_from_attention_colsum(cuda, monkeypatch, H, HKV, D, S):
    """A biased QKV projection feeding K8 packed attention: the backward kernels' dQKV column sums
    become the projection's bias gradient (no column-sum pass) -- equal to the fp32 reference."""
    import madnn

    calls = []
    real = madnn.ops.bias_grad
    monkeypatch.setattr(madnn.ops, "bias_grad", lambda *a, **k: calls.append(1) or real(*a, **k))
    torch.manual_seed(9)
    B, E = 2, 256
    x = torch.randn(B, S, E, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn((H + 2 * HKV) * D, E, device=cuda) * E ** -0.5).bfloat16().requires_grad_()
    b = (torch.randn((H + 2 * HKV) * D, device=cuda) * 0.1).bfloat16().requires_grad_()
    g = torch.randn(B, S, H, D, device=cuda)
    qkv = madnn.ops.linear(x, w, b).view(B, S, H + 2 * HKV, D)
    o = madnn.ops.attention_qkvpacked(qkv, H, HKV, causal=True)
    (o.float() * g).sum().backward()
    assert not calls, "the QKV projection ran its own bias column-sum pass"
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
    qf = torch.nn.functional.linear(xf, wf, bf).view(B, S, H + 2 * HKV, D)
    q, k, v = qf.split([H, HKV, HKV], dim=2)
    (_ref(q, k, v, True, D ** -0.5) * g).sum().backward()
    assert _rel(b.grad, bf.grad) < 2e-2 and _rel(w.grad, wf.grad) < 2e-2 and _rel(x.grad, xf.grad) < 2e-2


# madnn_attn_tune keys (attn.hip): 7 = dK/dV on the LDS-DMA ring, 8 = forward on it; value 0 forces the
# register-staged kernels that otherwise serve only ragged lengths and D = 128
_VARIANTS = [(7, 0), (8, 0)]


@pytest.mark.parametrize("key,value", _VARIANTS)
@pytest.mark.parametrize("B,S,H,HKV,D,causal", [(1, 256, 4, 2, 64, True), (2, 192, 2, 2, 64, False)])
def test_attention_tunable_variants_match_reference(cuda, key, value, B, S, H, HKV, D, causal):
    import ctypes

    assert ops.load_kernels()
    knob = ctypes.CDLL(str(ops.kernels_path())).madnn_attn_tune
    old = knob(key, value)
    assert old >= 0
    try:
        torch.manual_seed(1)
        q = torch.randn(B, S, H, D, device=cuda).bfloat16().requires_grad_(True)
        k = torch.randn(B, S, HKV, D, device=cuda).bfloat16().requires_grad_(True)
        v = torch.randn(B, S, HKV, D, device=cuda).bfloat16().requires_grad_(True)
        o = ops.attention(q, k, v, causal=causal)
        do = torch.randn_like(o)
        o.backward(do)
        torch.cuda.synchronize()
    finally:
        knob(key, old)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = _ref(qr, kr, vr, causal, D ** -0.5)
    orf.backward(do.float())
    assert _rel(o, orf) < 1e-2
    for g, gr, name in ((q.grad, qr.grad, "dq"), (k.grad, kr.grad, "dk"), (v.grad, vr.grad, "dv")):
        assert _rel(g, gr) < 2e-2, name


@pytest.mark.parametrize("S,D", [(512, 64), (320, 64), (384, 128)])
@pytest.mark.parametrize("order", ["grow", "shrink"])
def test_attention_online_softmax_rescale_branch(cuda, S, D, order):
    """The forward's lazy rescale (a row's reference moves only when its max grows by more than the
    slack) on inputs that force it (cdna_hip_programming.md rule 26): 'grow' multiplies the keys of
    the second half by 6 so every row's max jumps several tiles in; 'shrink' puts the large keys
    first, so later tiles sit far below the reference (exp2 of large negatives).  Against fp32."""
    torch.manual_seed(5)
    B, H = 1, 2
    q = torch.randn(B, S, H, D, device=cuda)
    k = torch.randn(B, S, H, D, device=cuda)
    v = torch.randn(B, S, H, D, device=cuda)
    big = slice(S // 2, S) if order == "grow" else slice(0, S // 2)
    k[:, big] *= 6.0
    q, k, v = (t.bfloat16().requires_grad_(True) for t in (q, k, v))
    for causal in (True, False):
        o = ops.attention(q, k, v, causal=causal)
        do = torch.randn_like(o)
        gq, gk, gv = torch.autograd.grad(o, (q, k, v), do)
        qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
        orf = _ref(qr, kr, vr, causal, D ** -0.5)
        rq, rk, rv = torch.autograd.grad(orf, (qr, kr, vr), do.float())
        assert torch.isfinite(o.float()).all()
        assert _rel(o, orf) < 1.5e-2, (causal, _rel(o, orf))
        for g, gr, name in ((gq, rq, "dq"), (gk, rk, "dk"), (gv, rv, "dv")):
            assert _rel(g, gr) < 3e-2, (causal, name, _rel(g, gr))
