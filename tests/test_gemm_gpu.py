"""K12 MFMA GEMM (madnn/ops/csrc/gemm.hip) against a plain PyTorch fp32 reference.

Shapes cover full 256x256 tiles, ragged M and N edges, a single K step and deep reductions;
the epilogue variants (fp32 / bf16 bias, tanh-GELU with the pre-activation saved, residual)
and the data gradient with in-place accumulation."""
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


SHAPES = [(512, 256, 64), (300, 200, 128), (1024, 384, 1024), (777, 1032, 320), (4096, 1024, 4096)]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_linear_fwd_plain(M, N, K):
    m = _ops()
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    y, aux = m.linear_fwd(x, w, None, None, 0, False)
    ref = x.float() @ w.float().t()
    assert y.shape == (M, N) and aux.numel() == 0
    assert _rel(y, ref) < 6e-3
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("bias_dtype", [torch.float32, torch.bfloat16])
def test_linear_fwd_bias_gelu_aux(bias_dtype):
    m = _ops()
    M, N, K = 1000, 768, 512
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(2, M // 2, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g).to(bias_dtype)
    y, pre = m.linear_fwd(x, w, b, None, 1, True)
    ref_pre = x.float() @ w.float().t() + b.float()
    assert y.shape == (2, M // 2, N) and pre.shape == y.shape
    torch.testing.assert_close(pre.float(), ref_pre, atol=3e-2, rtol=2e-2)
    # GELU is applied to the bf16-rounded pre-activation, exactly as the unfused graph does
    torch.testing.assert_close(y.float(), F.gelu(pre.float(), approximate="tanh"), atol=1e-2, rtol=1e-2)


def test_linear_fwd_residual():
    m = _ops()
    M, N, K = 640, 512, 256
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    y, _ = m.linear_fwd(x, w, b, r, 0, False)
    ref = (x.float() @ w.float().t() + b).bfloat16().float() + r.float()
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M,N,K", [(512, 256, 256), (300, 192, 200), (2048, 3072, 1024), (1000, 1024, 4096)])
def test_linear_dgrad(M, N, K):
    m = _ops()
    g = torch.Generator(device="cuda").manual_seed(M * 3 + K)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * N ** -0.5).bfloat16()
    dx = m.linear_dgrad(dy, w, None, False)
    ref = dy.float() @ w.float()
    assert _rel(dx, ref) < 6e-3
    torch.testing.assert_close(dx.float(), ref, atol=3e-2, rtol=2e-2)
    # accumulate in place into an existing gradient (beta = 1)
    acc = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    want = (ref.bfloat16().float() + acc.float())
    out = m.linear_dgrad(dy, w, acc, True)
    assert out.data_ptr() == acc.data_ptr()
    torch.testing.assert_close(acc.float(), want, atol=4e-2, rtol=2e-2)


def test_linear_asymmetric_exact():
    """Small-integer operands: every product and sum is exact in fp32, so K12 must match the
    once-rounded reference bit for bit (catches transposed fragments / swapped output indices)."""
    m = _ops()
    M, N, K = 513, 320, 192
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randint(-3, 4, (M, K), device="cuda", generator=g).bfloat16()
    w = torch.randint(-2, 3, (N, K), device="cuda", generator=g).bfloat16()
    w[:, 0] = torch.arange(N, device="cuda").remainder(7).bfloat16()  # asymmetric
    y, _ = m.linear_fwd(x, w, None, None, 0, False)
    assert torch.equal(y, (x.float() @ w.float().t()).bfloat16())
    dy = torch.randint(-3, 4, (M, N), device="cuda", generator=g).bfloat16()
    dx = m.linear_dgrad(dy, w, None, False)
    assert torch.equal(dx, (dy.float() @ w.float()).bfloat16())


# ---- weight gradient: dW[N, K] = dy[M, N]^T x[M, K], split along the M tokens
WGRAD_SHAPES = [(256, 256, 64, 1), (4096, 1024, 1024, 0), (2048, 3072, 1024, 5), (1024, 200, 520, 3),
                (8192, 1032, 4096, 0), (64, 64, 64, 1)]


# K12 (8 waves), K12W (4 waves, 32x32x16), K12W16 (4 waves, 16x16x32: tokens a multiple of 128)
@pytest.mark.parametrize("kernel", ["linear_wgrad", "linear_wgrad4", "linear_wgrad4h"])
@pytest.mark.parametrize("M,N,K,splits", WGRAD_SHAPES + [(64 * 37, 136, 1000, 7), (64 * 20, 520, 264, 40),
                                         (128 * 37, 136, 1000, 7)])
def test_linear_wgrad_split_k(M, N, K, splits, kernel):
    """The weight-gradient kernels against fp32, with ragged N / K tiles, odd K-tile counts (K12W
    runs its K loop in pairs; K12W16 gives every split an even count) and more splits than K tiles
    per split (empty splits write zeros)."""
    if kernel == "linear_wgrad4h" and M % 128:
        pytest.skip("K12W16 takes token counts that are multiples of 128 (the binding refuses others)")
    m = _ops()
    wgrad = getattr(m, kernel)
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    dw = wgrad(dy, x, None, False, splits)
    ref = dy.float().t() @ x.float()
    assert dw.shape == (N, K) and dw.dtype == torch.bfloat16
    assert _rel(dw, ref) < 6e-3, (M, N, K, splits)
    # accumulate into an existing gradient (a second backward before the optimizer step)
    base = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    out = base.clone()
    wgrad(dy, x, out, True, splits)
    assert _rel(out, ref + base.float()) < 6e-3


def test_linear_wgrad4h_refuses_odd_token_tiles():
    m = _ops()
    dy = torch.randn(64 * 3, 256, device="cuda").bfloat16()
    x = torch.randn(64 * 3, 256, device="cuda").bfloat16()
    with pytest.raises(RuntimeError, match="multiple of 128"):
        m.linear_wgrad4h(dy, x, None, False, 0)


def test_linear_wgrad_splits_heuristic_fills_the_gpu():
    m = _ops()
    # GPT-2 medium at 64 x 1024 tokens: 16 (proj) .. 64 (c_fc) output tiles -> split the tokens
    for N, K in ((1024, 1024), (3072, 1024), (4096, 1024), (1024, 4096)):
        tiles = (N // 256) * (K // 256)
        sp = m.wgrad_splits(65536, N, K)
        assert sp >= 2 and 192 <= tiles * sp, (N, K, sp)  # >= 3/4 of the 256 CUs busy
    assert m.wgrad_splits(64, 1024, 1024) == 1  # nothing to split
