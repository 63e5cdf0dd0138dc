// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels.
//
// Everything in csrc/ is written directly for gfx950: 64-lane wavefronts,
// MFMA matrix cores (v_mfma_f32_32x32x16_bf16 / 16x16x32_bf16), 160 KiB LDS.
// There is no CUDA path and no platform #ifdef: this is CDNA4 code.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace dta {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
// Plain cast lowers to v_cvt_pk_bf16_f32 (RNE, NaN-preserving) at -O3.
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// Four floats -> bf16x4 through two-wide vector conversions (one v_cvt_pk_bf16_f32
// per pair; the scalar casts above pair their results up with an extra v_perm)
__device__ __forceinline__ bf16x4 pk4_bf16(float a, float b, float c, float d) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 h2 __attribute__((ext_vector_type(2)));
  const h2 lo = __builtin_convertvector(f2{a, b}, h2);
  const h2 hi = __builtin_convertvector(f2{c, d}, h2);
  return bf16x4{lo[0], lo[1], hi[0], hi[1]};
}

// ReLU as one integer max on the bits (negative floats are negative int32s; -0 -> +0):
// x > 0 ? x : 0 compiles to a canonicalising v_max_f32 pair
__device__ __forceinline__ float relu1(float x) {
  return __builtin_bit_cast(float, max(__builtin_bit_cast(int, x), 0));
}

// 8-element vector load/store with fp32 conversion (16-byte bf16 / 32-byte fp32)
__device__ __forceinline__ void load8(const bf16* p, float* f) {
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = bf2f(v[j]);
}
__device__ __forceinline__ void store8(bf16* p, const float* f) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(f[j]);
  *reinterpret_cast<bf16x8*>(p) = v;
}

__device__ __forceinline__ void load8(const float* p, float* f) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void store8(float* p, const float* f) {
  reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
}

// DPP move of `v` (lanes outside ROWMASK keep `old`): a VALU modifier, a few
// cycles, where __shfl_xor is an LDS-path ds_bpermute with ~100+ cycles of
// latency per step -- six of those sat on the per-step critical path of the
// persistent MLP loop's loss phase.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_mov(float old, float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                               CTRL, ROWMASK, 0xf, false));
}

// Full-wave sum / max, result in every lane (requires all 64 lanes active):
// quad swaps, half-row and row mirrors give each 16-lane row its total; row
// broadcasts 15 and 31 chain the rows into lane 63, which is read back.
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_mov<0xB1, 0xf>(0.f, v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E, 0xf>(0.f, v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141, 0xf>(0.f, v);  // row_half_mirror
  v += dpp_mov<0x140, 0xf>(0.f, v);  // row_mirror
  v += dpp_mov<0x142, 0xa>(0.f, v);  // row_bcast:15 -> rows 1, 3
  v += dpp_mov<0x143, 0xc>(0.f, v);  // row_bcast:31 -> rows 2, 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1, 0xf>(v, v));
  v = fmaxf(v, dpp_mov<0x4E, 0xf>(v, v));
  v = fmaxf(v, dpp_mov<0x141, 0xf>(v, v));
  v = fmaxf(v, dpp_mov<0x140, 0xf>(v, v));
  v = fmaxf(v, dpp_mov<0x142, 0xa>(v, v));
  v = fmaxf(v, dpp_mov<0x143, 0xc>(v, v));
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// Sum over the 32 lanes that share one half of the wave (lanes 0-31 or 32-63).
__device__ __forceinline__ float half_wave_sum(float v) {
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Row index of accumulator register `reg` for v_mfma_f32_32x32x16_bf16
// (column = lane & 31).  cdna_hip_programming.md §3.
__device__ __forceinline__ int mfma32_row(int reg, int lane) {
  return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
}

__device__ __forceinline__ f32x16 mfma32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 mfma16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Column sums of fp32 [nrows, C] partials for columns c0 .. c0+31, by one
// 256-thread workgroup: 32 columns x 8 row groups, 8 independent loads in
// flight per thread, LDS reduce.  out: bf16 and/or f32 (nullptr: skip).
__device__ __forceinline__ void colsum_block(const float* __restrict__ part, int nrows, int C, int c0,
                                             bf16* __restrict__ out_bf16, float* __restrict__ out_f32) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c = c0 + cl;
  float s = 0.f;
  if (c < C) {
    int r = rg;
    for (; r + 56 < nrows; r += 64) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(r + 8 * u) * C + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; r < nrows; r += 8) s += part[(int64_t)r * C + c];
  }
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += red[g][cl];
    if (out_bf16) out_bf16[c] = f2bf(t);
    if (out_f32) out_f32[c] = t;
  }
}

// XCD-aware bijective remap of a 1-D block id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): blocks that land on one XCD (b % 8 equal)
// get a contiguous chunk of the logical tile space so they share L2 panels.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nxcd = 8;
  if (nwg <= nxcd) return orig;
  const int q = nwg / nxcd, r = nwg % nxcd;
  const int xcd = orig % nxcd;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / nxcd;
}

// One global_load_lds_dwordx4: 64 lanes x 16 B from per-lane `gsrc` to the
// wave-uniform LDS address `lds_base` + 16 * lane.  Inline asm, not the
// builtin: with the builtin hipcc treats the DMA as a pending write to the
// LDS array and waits vmcnt(0) before the next ds_read of ANY buffer, which
// serialises the stage loads with the multiply.  The asm load is invisible to
// hipcc's counters: the kernel counts them itself (vm_wait below).
__device__ __forceinline__ void glds16(const void* gsrc, char* lds_base) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) char*)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(dst)
               : "memory");
}

// One LDS-DMA piece through a buffer descriptor: 64 lanes x 16 B from (descriptor base + voff + soff)
// to the wave-uniform LDS address `lds_base` + 16 * lane.  Against global_load_lds (a 64-bit flat
// address per lane, advanced by a 64-bit VALU add per piece and K-step) the lane supplies a 32-bit
// offset fixed for the whole K loop and the K-step moves the scalar soffset.
// `dst`: the wave-uniform LDS byte address itself (lds_addr of the staging array + offsets in
// scalar registers: no per-piece generic -> LDS pointer conversion with its null check)
__device__ __forceinline__ void bglds16(__amdgpu_buffer_rsrc_t rsrc, unsigned voff, unsigned soff, unsigned dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(dst), "s"(soff)
      : "memory");
}

// bglds16 without the M0 save / restore, for kernels that own M0 (no other M0 use in the loop: the
// compiler is told M0 is clobbered).  The restore right behind the load waited for the load to dispatch
// (it reads M0 then): with one wave per SIMD that wait sat in the MFMA stream (csrc/gemm_w4.hip).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // M0 is "reserved": the kernels using this have no other M0 use
__device__ __forceinline__ void bglds16_m0(__amdgpu_buffer_rsrc_t rsrc, unsigned voff, unsigned soff, unsigned dst) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
               :
               : "v"(voff), "s"(rsrc), "s"(dst), "s"(soff)
               : "memory", "m0");
}
#pragma clang diagnostic pop

// LDS byte address of a __shared__ object (wave-uniform)
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) char*)p);
}

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU_TANH = 2, ACT_SILU = 3 };

__device__ __forceinline__ float act_fwd(int act, float x) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_GELU_TANH: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      float t = tanhf(k0 * (x + k1 * x * x * x));
      return 0.5f * x * (1.f + t);
    }
    case ACT_SILU: return x / (1.f + __expf(-x));
    default: return x;
  }
}

// d act(x) / dx
__device__ __forceinline__ float act_bwd(int act, float x) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case ACT_GELU_TANH: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      float u = k0 * (x + k1 * x * x * x);
      float t = tanhf(u);
      float du = k0 * (1.f + 3.f * k1 * x * x);
      return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * du;
    }
    case ACT_SILU: {
      float s = 1.f / (1.f + __expf(-x));
      return s * (1.f + x * (1.f - s));
    }
    default: return 1.f;
  }
}

}  // namespace dta

#define DTA_HIP_CHECK(expr)                                                   \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) return _e;                                          \
  } while (0)
