// Shared (host <-> device) argument block of the K8 attention kernels.
#pragma once
#include <stdint.h>

extern "C" {

// All tensors bf16 except lse/delta (fp32).  q/k/v (and dq/dk/dv) are [B, S, heads, D]
// views with the last dim contiguous; any batch/seq/head strides (in elements) -- e.g.
// slices of one packed [B, S, H + 2*Hkv, D] QKV projection.  o/dout are [B, S, H, D]
// with strides o_*.  lse/delta are [B, H, S] fp32 (lse in log2 units of the scaled score).
struct MadnnAttnArgs {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  uint16_t* o;
  float* lse;
  const uint16_t* dout;
  uint16_t* dq;
  uint16_t* dk;
  uint16_t* dv;
  float* delta;
  int64_t q_sb, q_ss, q_sh;
  int64_t k_sb, k_ss, k_sh;
  int64_t v_sb, v_ss, v_sh;
  int64_t o_sb, o_ss, o_sh;
  int64_t dq_sb, dq_ss, dq_sh;
  int64_t dk_sb, dk_ss, dk_sh;
  int64_t dv_sb, dv_ss, dv_sh;
  int B, S, H, Hkv;
  float scale;       // softmax scale (1/sqrt(D) by default)
  float scale_log2;  // scale * log2(e)
  // backward, optional: per-workgroup column sums of the written dq / dk / dv (the packed QKV
  // projection's bias gradient before the final reduce): [B * ceil(S / 128)][(H + 2 Hkv) * D] fp32,
  // dq in columns [0, H D), dk in [H D, (H + Hkv) D), dv in [(H + Hkv) D, (H + 2 Hkv) D)
  float* cpart;
};

}
