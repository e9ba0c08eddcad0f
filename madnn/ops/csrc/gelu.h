// tanh-GELU forward / derivative on v_exp_f32 + v_rcp_f32, shared by the standalone GELU passes
// (K11, bias.hip) and the fused GEMM epilogues (K12, gemm.hip / gemmp.hip): one formula, so a
// fused epilogue rounds exactly as the unfused pass it replaces.
#pragma once

#include "common.h"

namespace madnn {

// On v_exp_f32 and v_rcp_f32 (1 ulp): libm tanhf is ~30 VALU per element with range branches, and at
// 32 elements per lane per row step the GELU backward pass was partly VALU-bound instead of HBM-bound
// (the libm and IEEE-division variants were measured and dropped, rounds 2-3).
// tanh-GELU through the logistic function: with u = k0 (x + k1 x^3),
//   gelu(x)  = 0.5 x (1 + tanh u) = x s,      s = sigmoid(2u) = 1 / (1 + 2^(-2u log2 e))
//   gelu'(x) = s + x s (1 - s) 2 u'(x),       2 u'(x) = 2 k0 (1 + 3 k1 x^2)
// The constants fold into the polynomials, so the forward is 5 VALU + v_exp + v_rcp per element
// and the backward 9 + the same two (the tanh form took ~11 / ~20 VALU: the streaming GELU passes
// sit close enough to the HBM roofline that their VALU work shows in the wall time).  x -> -inf
// gives s = 0 (2^+inf = inf, rcp(inf) = 0), x -> +inf gives s = 1 exactly.
__device__ __forceinline__ float gelu_sig_arg(float x, float x2) {
  // -2 u log2(e) = x (A + B x^2)
  constexpr float kA = -2.f * 0.7978845608028654f * 1.4426950408889634f;
  constexpr float kB = kA * 0.044715f;
  return x * fmaf(kB, x2, kA);
}

__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float e = __builtin_amdgcn_exp2f(gelu_sig_arg(x, x2));
  const float s = __builtin_amdgcn_rcpf(1.f + e);
  const float du = x * fmaf(2.f * k0 * 3.f * k1, x2, 2.f * k0);  // x 2u'(x)
  return fmaf(du * s, 1.f - s, s);
}

// y = gelu_tanh(x) = x sigmoid(2u) on v_exp / v_rcp: the standalone GELU forward pass after c_fc
// (hipBLASLt on gfx950 has no GELU epilogue that also returns the pre-activation the backward
// needs, bench/lt_probe.py).
__device__ __forceinline__ float gelu_tanh(float x) {
  const float e = __builtin_amdgcn_exp2f(gelu_sig_arg(x, x * x));
  return x * __builtin_amdgcn_rcpf(1.f + e);
}

}  // namespace madnn
