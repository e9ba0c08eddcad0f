"""K14 (RoPE on the packed QKV) and K15 (SwiGLU) against fp32 PyTorch references
(madnn/ops/csrc/glue.hip)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


@pytest.mark.parametrize("H,HKV,D,S", [(4, 4, 64, 96), (8, 2, 128, 200), (32, 8, 128, 64)])
def test_rope_qkv_kernel_matches_fp32(cuda, H, HKV, D, S):
    from madnn import ops
    from madnn.models.common import RotaryEmbedding

    assert ops.load_kernels()
    torch.manual_seed(0)
    rope = RotaryEmbedding(D, 500000.0, 256).to(cuda)
    B = 2
    qkv = torch.randn(B, S, H + 2 * HKV, D, device=cuda).bfloat16()
    ref = qkv.float().clone()
    ref[:, :, : H + HKV] = ops._rope_rotate(ref[:, :, : H + HKV], rope.cos, rope.sin, False).float()
    out = torch.ops.madnn.rope_qkv(qkv, rope.cos, rope.sin, H + HKV, False)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=1e-2)
    assert torch.equal(out[:, :, H + HKV:], qkv[:, :, H + HKV:])          # v untouched
    # the inverse rotation undoes the forward (to bf16 rounding)
    back = torch.ops.madnn.rope_qkv_(out.clone(), rope.cos, rope.sin, H + HKV, True)
    torch.testing.assert_close(back.float(), qkv.float(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M,I", [(257, 64), (1024, 1408), (64, 14336)])
def test_swiglu_kernels_match_fp32(cuda, M, I):
    from madnn import ops

    assert ops.load_kernels()
    torch.manual_seed(1)
    gu = (torch.randn(M, 2 * I, device=cuda) * 2).bfloat16().requires_grad_(True)
    h = ops.swiglu(gu)
    dh = torch.randn_like(h)
    h.backward(dh)
    gf = gu.detach().float().requires_grad_(True)
    g, u = gf.chunk(2, -1)
    hr = F.silu(g) * u
    hr.backward(dh.float())
    assert h.dtype == torch.bfloat16 and _rel(h, hr) < 1e-2
    assert _rel(gu.grad, gf.grad) < 1e-2


def test_llama_block_k14_k15_match_eager(cuda, monkeypatch):
    """A Llama block (GQA, RoPE, SwiGLU) on the fused path (K14 + K8 packed + K15 + residual in the
    down projection's epilogue) vs the same block with attention forced onto SDPA (the eager RoPE
    path) and the eager SwiGLU: outputs and every gradient agree."""
    from madnn import ops
    from madnn.models.llama import Llama, llama_config

    torch.manual_seed(2)
    model = Llama(llama_config("llama3-tiny", hidden=512, heads=4, kv_heads=2, intermediate=512, layers=2)).to(cuda)
    model = model.bfloat16()
    ids = torch.randint(0, model.config.vocab_size, (2, 128), device=cuda)
    loss = model.loss_fn(model(ids), ids)
    loss.backward()
    got = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    model.zero_grad()
    monkeypatch.setattr(ops, "attention_supported", lambda *a, **k: False)
    real = ops.swiglu
    monkeypatch.setattr(ops, "swiglu", lambda gu: real(gu.float()).to(gu.dtype))
    loss2 = model.loss_fn(model(ids), ids)
    loss2.backward()
    torch.testing.assert_close(loss.float(), loss2.float(), atol=2e-2, rtol=2e-2)
    for n, p in model.named_parameters():
        assert _rel(got[n], p.grad) < 5e-2, (n, _rel(got[n], p.grad))


def test_misaligned_inputs_are_refused_or_rerouted(cuda):
    """K14 / K15 move 16 bytes per lane: a contiguous slice that starts off a 16-byte boundary is
    refused by the bindings (never a misaligned vector access) and handled by ``ops`` (an aligned
    copy for RoPE, the eager path for SwiGLU) with the right result."""
    from madnn import ops
    from madnn.models.common import RotaryEmbedding

    assert ops.load_kernels()
    torch.manual_seed(3)
    buf = torch.randn(1 + 64 * 32, device=cuda).bfloat16()
    gu = buf[1:].view(64, 32)                      # 2-byte offset: misaligned, contiguous
    assert gu.is_contiguous() and gu.data_ptr() % 16
    with pytest.raises(RuntimeError, match="16-byte aligned"):
        torch.ops.madnn.swiglu_fwd(gu)
    g, u = gu.float().chunk(2, -1)
    assert _rel(ops.swiglu(gu), F.silu(g) * u) < 1e-2
    D, H, HKV, S = 64, 2, 1, 16
    rope = RotaryEmbedding(D, 10000.0, 64).to(cuda)
    qb = torch.randn(8 + 2 * S * (H + 2 * HKV) * D, device=cuda).bfloat16()
    qkv = qb[8 * 0 + 1: 1 + 2 * S * (H + 2 * HKV) * D].view(2, S, H + 2 * HKV, D)
    assert qkv.data_ptr() % 16
    with pytest.raises(RuntimeError, match="16-byte aligned"):
        torch.ops.madnn.rope_qkv(qkv, rope.cos, rope.sin, H + HKV, False)
    ref = qkv.float().clone()
    ref[:, :, : H + HKV] = ops._rope_rotate(ref[:, :, : H + HKV], rope.cos, rope.sin, False).float()
    torch.testing.assert_close(ops.rope_qkv(qkv, rope.cos, rope.sin, H + HKV).float(), ref, atol=2e-2, rtol=1e-2)
