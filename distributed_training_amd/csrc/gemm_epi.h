// Shared pieces of the hand-written bf16 GEMMs (csrc/gemm_k64.hip, csrc/gemm_w4.hip): the argument
// block, the fused epilogues (bias, GELU with dual store, GELU-derivative, residual) and the wait /
// barrier primitives of their LDS-DMA pipelines.
#pragma once

#include "common.h"

namespace dta {
namespace k64 {

constexpr int BK = 64;
constexpr int kGroupM = 8;

// EPI_DSWIGLU (the input gradient of silu(a) * b through the down projection, Llama's SwiGLU MLP): the
// product is g = d(silu(a) b); res holds the rows [a | b] and c receives [da | db], both 2N wide (N = the
// GEMM's N = the MLP's hidden width): da = g b s (1 + a (1 - s)), db = g a s, s = sigmoid(a)
enum Epi : int { EPI_NONE = 0, EPI_GELU = 2, EPI_DGELU = 16, EPI_RES = 32, EPI_DSWIGLU = 64 };

struct Args {
  const bf16* a;
  const bf16* b;
  bf16* c;          // bf16 output (EPI_GELU with c2: the pre-activation)
  bf16* c2;         // EPI_GELU: the activation gelu(c) (nullptr: c holds the activation)
  float* c32;       // fp32 output instead of c (EPI_NONE only)
  const bf16* bias; // [N] or nullptr
  const bf16* res;  // EPI_DGELU: the GELU input; EPI_RES: added after rounding; EPI_DSWIGLU: [a | b] rows
  int64_t lda, ldb, ldc, ldc2, ldr;
  int M, N, K;
  int tiles_m, tiles_n;
  float alpha;
  int epi;
  bf16* db;  // weight-gradient groups: the bias gradient db[m] = sum_k A(m, k) (nullptr: none)
  const float* alpha_dev;  // nullptr, or a device scalar multiplying alpha (a loss scale known only on the GPU)
#if defined(DTA_K64_STAMP) || defined(DTA_K64_TIMELINE)
  unsigned long long* stamps;  // diagnostic build only: per-wave cycle sums of the two-phase loop's segments
#endif
};

// GELU (tanh form) as x * sigmoid(2u): one v_exp_f32 + one v_rcp_f32 instead of tanhf
__device__ __forceinline__ float gelu_fast(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  return x * __frcp_rn(1.f + __expf(-2.f * u));
}
__device__ __forceinline__ float gelu_grad_fast(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  const float s = __frcp_rn(1.f + __expf(-2.f * u));  // sigmoid(2u) = (1 + tanh u) / 2
  // d/dx [x s] = s + x s (1 - s) 2 du/dx
  return s + 2.f * x * s * (1.f - s) * k0 * (1.f + 3.f * k1 * x * x);
}

// ---- shared epilogue: bias of columns n .. n+3, and one lane's four accumulators (row m, columns n .. n+3) ----
__device__ __forceinline__ void load_bias4(const Args& g, int n, float (&bv)[4]) {
  bv[0] = bv[1] = bv[2] = bv[3] = 0.f;
  if (g.bias) {
    const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(g.bias + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = bf2f(b4[r]);
  }
}

// The bf16 values of output `which` (0: c, 1: c2 of the GELU dual store) at row m, columns n .. n+3 -- the
// fused epilogue of store4 below without the store (the LDS-staged epilogue of csrc/gemm_w4.hip stores them)
__device__ __forceinline__ float alpha_of(const Args& g) { return g.alpha_dev ? g.alpha * *g.alpha_dev : g.alpha; }

__device__ __forceinline__ bf16x4 val4(const Args& g, int m, int n, const f32x4& acc, const float (&bv)[4], int which) {
  float v[4];
  const float al = alpha_of(g);
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = fmaf(acc[r], al, bv[r]);
  if (g.epi == EPI_GELU) {
    if (g.c2) {
      const bf16x4 h4 = pk4_bf16(v[0], v[1], v[2], v[3]);
      if (which == 0) return h4;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = gelu_fast(bf2f(h4[r]));
      return pk4_bf16(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = gelu_fast(v[r]);
  } else if (g.epi == EPI_DGELU) {
    const bf16x4 h4 = *reinterpret_cast<const bf16x4*>(g.res + (int64_t)m * g.ldr + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= gelu_grad_fast(bf2f(h4[r]));
  } else if (g.epi == EPI_RES) {
    const bf16x4 r4 = *reinterpret_cast<const bf16x4*>(g.res + (int64_t)m * g.ldr + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = bf2f(f2bf(v[r])) + bf2f(r4[r]);
  }
  return pk4_bf16(v[0], v[1], v[2], v[3]);
}

// val4 of the EPI_DGELU / EPI_RES epilogues with the four res values given (read by the caller: the
// LDS-staged epilogue of csrc/gemm_k64.hip stages the res tile with whole-row loads first)
__device__ __forceinline__ bf16x4 val4_res(const Args& g, const f32x4& acc, const float (&bv)[4], const bf16x4 r4) {
  float v[4];
  const float al = alpha_of(g);
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = fmaf(acc[r], al, bv[r]);
  if (g.epi == EPI_DGELU) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= gelu_grad_fast(bf2f(r4[r]));
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = bf2f(f2bf(v[r])) + bf2f(r4[r]);
  }
  return pk4_bf16(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ void store4(const Args& g, int m, int n, const f32x4& acc, const float (&bv)[4]) {
  float v[4];
  const float al = alpha_of(g);
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = fmaf(acc[r], al, bv[r]);
  if (g.c32) {
    *reinterpret_cast<float4*>(g.c32 + (int64_t)m * g.ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
    return;
  }
  if (g.epi == EPI_GELU) {
    if (g.c2) {  // dual store: pre-activation h (for the backward) and gelu(h) (the next GEMM's input)
      const bf16x4 h4 = pk4_bf16(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<bf16x4*>(g.c + (int64_t)m * g.ldc + n) = h4;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = gelu_fast(bf2f(h4[r]));  // gelu of the stored (rounded) h
      *reinterpret_cast<bf16x4*>(g.c2 + (int64_t)m * g.ldc2 + n) = pk4_bf16(v[0], v[1], v[2], v[3]);
      return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = gelu_fast(v[r]);
  } else if (g.epi == EPI_DGELU) {  // dgrad through the GELU: one rounding (of the product)
    const bf16x4 h4 = *reinterpret_cast<const bf16x4*>(g.res + (int64_t)m * g.ldr + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= gelu_grad_fast(bf2f(h4[r]));
  } else if (g.epi == EPI_RES) {  // residual stream: round(round(linear) + res), as two bf16 ops give
    const bf16x4 r4 = *reinterpret_cast<const bf16x4*>(g.res + (int64_t)m * g.ldr + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = bf2f(f2bf(v[r])) + bf2f(r4[r]);
  }
  *reinterpret_cast<bf16x4*>(g.c + (int64_t)m * g.ldc + n) = pk4_bf16(v[0], v[1], v[2], v[3]);
}

// Grouped weight gradients: several problems' tiles in ONE launch (csrc/gemm_k64.hip, csrc/gemm_w4.hip)
constexpr int kGroupMax = 16;
struct GroupArgs {
  int n;
  int tile_start[kGroupMax + 1];
  Args p[kGroupMax];
};

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void bar() { asm volatile("s_barrier" ::: "memory"); }

}  // namespace k64
}  // namespace dta
