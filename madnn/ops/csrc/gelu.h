// GELU forward / derivative on v_exp_f32 + v_rcp_f32, shared by the standalone GELU passes (K11,
// bias.hip) and the fused GEMM epilogues (K12, gemm.hip / gemmp.hip): one formula per kind, so a
// fused epilogue rounds exactly as the unfused pass it replaces.  Two kinds (template GK):
// kGeluTanh (GPT-2's tanh approximation) and kGeluErf (BERT's exact erf form).
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

// exact (erf) GELU: gelu(x) = x Phi(x), Phi(x) = 0.5 (1 + erf(x / sqrt 2)),
// gelu'(x) = Phi(x) + x phi(x), phi(x) = exp(-x^2 / 2) / sqrt(2 pi).
// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below bf16's 2^-9): for z >= 0,
// erf(z) = 1 - t (a1 + t (a2 + t (a3 + t (a4 + t a5)))) e^(-z^2), t = 1 / (1 + p z); the e^(-z^2)
// is phi's exponential too, so the derivative costs no second exp.
struct ErfParts {
  float phi_cdf;   // Phi(x)
  float phi_pdf;   // phi(x)
};

__device__ __forceinline__ ErfParts gelu_erf_parts(float x) {
  constexpr float kP = 0.3275911f, kA1 = 0.254829592f, kA2 = -0.284496736f, kA3 = 1.421413741f,
                  kA4 = -1.453152027f, kA5 = 1.061405429f;
  constexpr float kRs2 = 0.7071067811865476f, kLog2e = 1.4426950408889634f, kRs2pi = 0.3989422804014327f;
  const float z = fabsf(x) * kRs2;
  const float t = __builtin_amdgcn_rcpf(fmaf(kP, z, 1.f));
  const float e = __builtin_amdgcn_exp2f(-z * z * kLog2e);   // e^(-z^2) = e^(-x^2 / 2)
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, kA5, kA4), kA3), kA2), kA1);
  const float erf_abs = 1.f - poly * e;                        // erf(|x| / sqrt 2)
  const float erf_x = x < 0.f ? -erf_abs : erf_abs;
  return {0.5f * (1.f + erf_x), kRs2pi * e};
}

__device__ __forceinline__ float gelu_erf(float x) { return x * gelu_erf_parts(x).phi_cdf; }

__device__ __forceinline__ float gelu_erf_grad(float x) {
  const ErfParts q = gelu_erf_parts(x);
  return fmaf(x, q.phi_pdf, q.phi_cdf);
}

enum GeluKind : int { kGeluTanh = 1, kGeluErf = 2 };

template <int GK>
__device__ __forceinline__ float gelu_act(float x) {
  if constexpr (GK == kGeluErf) return gelu_erf(x);
  else return gelu_tanh(x);
}

template <int GK>
__device__ __forceinline__ float gelu_act_grad(float x) {
  if constexpr (GK == kGeluErf) return gelu_erf_grad(x);
  else return gelu_tanh_grad(x);
}

}  // namespace madnn
