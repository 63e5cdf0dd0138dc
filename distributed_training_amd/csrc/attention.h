// Flash-attention launch arguments, shared by csrc/attention.hip (device
// code) and csrc/bindings.cpp (host checks).  Plain C types only: the host
// translation unit is compiled by g++.
#pragma once
#include <cstdint>

namespace dta {

struct AttnArgs {
  const void* q;        // [B, S, H, D]   bf16, arbitrary batch / token strides, head stride D
  const void* k;        // [B, S, Hkv, D]
  const void* v;        // [B, S, Hkv, D]
  void* o;              // [B, S, H, D]
  float* lse;           // [B, H, S] natural-log LSE of the scaled scores
  const void* dout;     // [B, S, H, D]
  float* delta;         // [B, H, S]  rowsum(dO * O)
  void* dq;             // [B, S, H, D]   bf16
  void* dk;             // [B, S, Hkv, D] bf16
  void* dv;             // [B, S, Hkv, D] bf16
  int64_t q_sb, q_ss, k_sb, k_ss, v_sb, v_ss;   // batch / token strides (elements)
  int64_t o_sb, o_ss, do_sb, do_ss;
  int64_t dq_sb, dq_ss, dk_sb, dk_ss, dv_sb, dv_ss;
  int B, S, H, Hkv;
  float scale;
  // backward only, nullptr = none: RoPE tables [S, D/2] (fp32) of the forward's rotation -- dQ / dK leave the
  // kernels inverse-rotated (the gradient of the pre-rotation q / k), in fp32 before their rounding
  const float* rcos;
  const float* rsin;
};

}  // namespace dta
