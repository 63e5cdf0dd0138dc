// Memory-bound transformer ops for gfx950: LayerNorm / RMSNorm (fwd + bwd),
// GELU(tanh), SwiGLU, rotary embedding, fused softmax-cross-entropy.
//
// All bf16 activations are moved with 16-byte vector accesses (8 x bf16 per
// lane, cdna_hip_programming.md Guideline 13); statistics in fp32.  One wave
// (64 lanes) per row for the row-wise ops: a row of C <= 8192 elements lives in
// registers (C / 512 vectors per lane), so the backward needs no second read.
#include "common.h"

namespace dta {

// ---------------------------------------------------------------- norms
// NV = vectors of 8 per lane (C = 512 * NV).  RMS: no mean, no bias.
template <int NV, bool RMS>
// res != nullptr: fused residual add, x_new = bf16(x + res) is written to
// xsum and normalised (the pre-LN block's "x = x + sublayer(x); y = LN(x)").
__global__ void __launch_bounds__(256) norm_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                       const bf16* __restrict__ bias, bf16* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int64_t N, int C, float eps, const bf16* __restrict__ res,
                                                       bf16* __restrict__ xsum) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const bf16* xr = x + row * C;
  float v[NV][8];
  float s = 0.f;
  // gamma / beta requested with the row (not after the two reductions): each wave handles one row of
  // the single round of rows, so a load issued late is a whole extra L2 round trip on its chain
  // (NV <= 4, GPT-2 sized rows: Llama-3 rows (NV 8) already stream at ~5.3 TB/s, and the hoisted vectors
  // would cost them occupancy)
  constexpr bool HOIST = NV <= 4;
  bf16x8 wraw[NV], braw[NV];
  auto load_wb = [&](int i) {
    const int c = min((i * 64 + lane) * 8, C - 8);
    wraw[i] = *reinterpret_cast<const bf16x8*>(w + c);
    if (!RMS) braw[i] = *reinterpret_cast<const bf16x8*>(bias + c);
  };
  if constexpr (HOIST) {
#pragma unroll
    for (int i = 0; i < NV; ++i) load_wb(i);
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (c < C) {
      load8(xr + c, v[i]);
      if (res) {
        float r[8];
        load8(res + row * C + c, r);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o[j] = f2bf(v[i][j] + r[j]);
          v[i][j] = bf2f(o[j]);  // normalise exactly the bf16 value that is stored
        }
        *reinterpret_cast<bf16x8*>(xsum + row * C + c) = o;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[i][j];
  }
  float mean = 0.f;
  if (!RMS) mean = wave_sum(s) / C;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (c < C)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        ss += d * d;
      }
  }
  const float rstd = rsqrtf(wave_sum(ss) / C + eps);
  if (lane == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
  bf16* yr = y + row * C;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (c < C) {
      if constexpr (!HOIST) load_wb(i);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * bf2f(wraw[i][j]) + (RMS ? 0.f : bf2f(braw[i][j]));
      store8(yr + c, o);
    }
  }
}

// dx per row; per-workgroup partial dgamma / dbeta sums into fp32 [nblk][C]
template <int NV, bool RMS>
__global__ void __launch_bounds__(256) norm_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                       const bf16* __restrict__ w, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, bf16* __restrict__ dx,
                                                       float* __restrict__ dw_part, float* __restrict__ db_part,
                                                       int64_t N, int C, int rows_per_block,
                                                       const bf16* __restrict__ dres) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float dwacc[NV][8], dbacc[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[i][j] = dbacc[i][j] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t rend = min(r0 + rows_per_block, N);
  // one row ahead in flight: the next row's x / dy / dres (raw bf16) and stats
  // are loaded before this row's reductions, so a wave's rows do not serialise
  // on load latency (the kernel is latency-, not bandwidth-bound at C = 768)
  bf16x8 xn[NV], dn[NV], rn[NV];
  float mun = 0.f, rsn = 0.f;
  auto fetch = [&](int64_t row) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = min((i * 64 + lane) * 8, C - 8);  // clamped: lanes past C re-read a valid chunk, unused
      xn[i] = *reinterpret_cast<const bf16x8*>(x + row * C + c);
      dn[i] = *reinterpret_cast<const bf16x8*>(dy + row * C + c);
      if (dres) rn[i] = *reinterpret_cast<const bf16x8*>(dres + row * C + c);
    }
    mun = RMS ? 0.f : mean[row];
    rsn = rstd[row];
  };
  float wv[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) load8(w + min((i * 64 + lane) * 8, C - 8), wv[i]);
  if (r0 + wave < rend) fetch(r0 + wave);
  for (int64_t row = r0 + wave; row < rend; row += 4) {
    const float mu = mun, rs = rsn;
    bf16x8 xc[NV], dc[NV], rc[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      xc[i] = xn[i];
      dc[i] = dn[i];
      if (dres) rc[i] = rn[i];
    }
    if (row + 4 < rend) fetch(row + 4);
    float xh[NV][8], g[NV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (c < C) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xv = bf2f(xc[i][j]), dv = bf2f(dc[i][j]);
          xh[i][j] = (xv - mu) * rs;
          g[i][j] = dv * wv[i][j];
          s1 += g[i][j];
          s2 += g[i][j] * xh[i][j];
          dwacc[i][j] += dv * xh[i][j];
          dbacc[i][j] += dv;
        }
      }
    }
    const float m1 = RMS ? 0.f : wave_sum(s1) / C;
    const float m2 = wave_sum(s2) / C;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      if (c < C) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (g[i][j] - m1 - xh[i][j] * m2);
        if (dres) {  // gradient arriving on the residual stream (fused accumulate)
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += bf2f(rc[i][j]);
        }
        store8(dx + row * C + c, o);
      }
    }
  }
  // reduce the 4 waves' partials through LDS, one row of partials per block
  __shared__ float red[4][512 * 8 / 8];  // staged 512 floats at a time
  for (int i = 0; i < NV; ++i) {
    for (int pass = 0; pass < (RMS ? 1 : 2); ++pass) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // lanes hold 8 consecutive columns: column c = (i*64 + lane)*8 + j
        red[wave][lane * 8 + j] = pass == 0 ? dwacc[i][j] : dbacc[i][j];
      }
      __syncthreads();
      for (int e = threadIdx.x; e < 512; e += 256) {
        const int c = i * 512 + e;
        if (c < C) {
          const float v = red[0][e] + red[1][e] + red[2][e] + red[3][e];
          (pass == 0 ? dw_part : db_part)[(int64_t)blockIdx.x * C + c] = v;
        }
      }
      __syncthreads();
    }
  }
}

// Wide rows (C a multiple of 2048: Llama's 4096): one 256-thread workgroup per row, NVL = C / 2048
// 16-byte vectors per lane -- the one-wave-per-row form above needs C / 64 fp32 values of x-hat and
// g per lane plus the prefetched row (512 registers and scratch spills at C = 4096, one wave per
// SIMD).  The block walks its rows with the next row's loads in flight; the two per-row sums cross
// the four waves through a double-buffered LDS slot (one barrier per row); each thread owns its
// columns' dgamma / dbeta partials (no cross-wave reduction).
template <int NVL, bool RMS>
__global__ void __launch_bounds__(256) norm_bwd_wide_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                            const bf16* __restrict__ w, const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, bf16* __restrict__ dx,
                                                            float* __restrict__ dw_part, float* __restrict__ db_part,
                                                            int64_t N, int C, int rows_per_block,
                                                            const bf16* __restrict__ dres) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ float red[2][4][2];
  float dwacc[NVL][8], dbacc[NVL][8];
  bf16x8 wb[NVL];  // (kept packed)
#pragma unroll
  for (int i = 0; i < NVL; ++i) {
    wb[i] = *reinterpret_cast<const bf16x8*>(w + (i * 256 + tid) * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[i][j] = dbacc[i][j] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t rend = min(r0 + rows_per_block, N);
  bf16x8 xn[NVL], dn[NVL], rn[NVL];
  float mun = 0.f, rsn = 0.f;
  auto fetch = [&](int64_t row) {
#pragma unroll
    for (int i = 0; i < NVL; ++i) {
      const int64_t o = row * C + (i * 256 + tid) * 8;
      xn[i] = *reinterpret_cast<const bf16x8*>(x + o);
      dn[i] = *reinterpret_cast<const bf16x8*>(dy + o);
      if (dres) rn[i] = *reinterpret_cast<const bf16x8*>(dres + o);
    }
    mun = RMS ? 0.f : mean[row];
    rsn = rstd[row];
  };
  if (r0 < rend) fetch(r0);
  int par = 0;
  for (int64_t row = r0; row < rend; ++row, par ^= 1) {
    const float mu = mun, rs = rsn;
    bf16x8 xc[NVL], dc[NVL], rc[NVL];
#pragma unroll
    for (int i = 0; i < NVL; ++i) {
      xc[i] = xn[i];
      dc[i] = dn[i];
      if (dres) rc[i] = rn[i];
    }
    if (row + 1 < rend) fetch(row + 1);
    float xh[NVL][8], g[NVL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NVL; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xv = bf2f(xc[i][j]), dv = bf2f(dc[i][j]);
        xh[i][j] = (xv - mu) * rs;
        g[i][j] = dv * bf2f(wb[i][j]);
        s1 += g[i][j];
        s2 += g[i][j] * xh[i][j];
        dwacc[i][j] += dv * xh[i][j];
        dbacc[i][j] += dv;
      }
    if (!RMS) s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
      red[par][wave][0] = s1;
      red[par][wave][1] = s2;
    }
    __syncthreads();
    const float m1 = RMS ? 0.f : (red[par][0][0] + red[par][1][0] + red[par][2][0] + red[par][3][0]) / C;
    const float m2 = (red[par][0][1] + red[par][1][1] + red[par][2][1] + red[par][3][1]) / C;
#pragma unroll
    for (int i = 0; i < NVL; ++i) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rs * (g[i][j] - m1 - xh[i][j] * m2);
      if (dres) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += bf2f(rc[i][j]);
      }
      store8(dx + row * C + (i * 256 + tid) * 8, o);
    }
  }
#pragma unroll
  for (int i = 0; i < NVL; ++i) {
    float* pw = dw_part + (int64_t)blockIdx.x * C + (i * 256 + tid) * 8;
    *reinterpret_cast<float4*>(pw) = make_float4(dwacc[i][0], dwacc[i][1], dwacc[i][2], dwacc[i][3]);
    *reinterpret_cast<float4*>(pw + 4) = make_float4(dwacc[i][4], dwacc[i][5], dwacc[i][6], dwacc[i][7]);
    if (!RMS) {
      float* pb = db_part + (int64_t)blockIdx.x * C + (i * 256 + tid) * 8;
      *reinterpret_cast<float4*>(pb) = make_float4(dbacc[i][0], dbacc[i][1], dbacc[i][2], dbacc[i][3]);
      *reinterpret_cast<float4*>(pb + 4) = make_float4(dbacc[i][4], dbacc[i][5], dbacc[i][6], dbacc[i][7]);
    }
  }
}

// Column sums of one or two [nrows, C] partial sets (colsum_block): blocks
// [0, ceil(C/32)) finish set 0, the rest set 1 (e.g. a norm's dw and db in one launch).
__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ part0, const float* __restrict__ part1,
                                                     int nrows, int C, bf16* __restrict__ ob0, float* __restrict__ of0,
                                                     bf16* __restrict__ ob1, float* __restrict__ of1) {
  const int nb = (C + 31) / 32;
  if ((int)blockIdx.x < nb) colsum_block(part0, nrows, C, blockIdx.x * 32, ob0, of0);
  else colsum_block(part1, nrows, C, (blockIdx.x - nb) * 32, ob1, of1);
}

// Several partial sets finished in ONE launch (the norms' deferred gamma / beta gradients, ops/lm.py
// _NORM_DEFER): job j owns blocks [start[j], start[j + 1]), 32 columns each.  At GPT-2 size one norm's
// colsum_kernel is 48 workgroups and ~5 us, almost all launch and latency; a step has 25 of them.
struct ColsumJobs {
  static constexpr int kMax = 64;
  int n;
  int start[kMax + 1];
  const float* part[kMax];
  int nrows[kMax];
  int C[kMax];
  bf16* out[kMax];
};

__global__ void __launch_bounds__(256) colsum_batch_kernel(ColsumJobs jobs) {
  int j = 0;
  while (j + 1 < jobs.n && (int)blockIdx.x >= jobs.start[j + 1]) ++j;
  colsum_block(jobs.part[j], jobs.nrows[j], jobs.C[j], ((int)blockIdx.x - jobs.start[j]) * 32, jobs.out[j], nullptr);
}

// Partial column sums of a bf16 [N, C] matrix (bias gradients): a workgroup
// is 64 column lanes (8 columns each, 16-byte loads) x 4 row lanes over one
// row split; the [nsplit, C] fp32 partials are finished by colsum_kernel.
__global__ void __launch_bounds__(256) colsum_bf16_partial_kernel(const bf16* __restrict__ x, int64_t N, int C,
                                                                   int rows_per_split, float* __restrict__ part) {
  __shared__ float red[4][512];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + cl) * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_split;
  const int64_t r1 = min(r0 + rows_per_split, N);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < C) {
#pragma unroll 4
    for (int64_t r = r0 + rl; r < r1; r += 4) {
      float v[8];
      load8(x + r * C + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cl * 8 + j] = acc[j];
  __syncthreads();
  for (int e = threadIdx.x; e < 512; e += 256) {
    const int cc = blockIdx.x * 512 + e;
    if (cc < C) part[(int64_t)blockIdx.y * C + cc] = red[0][e] + red[1][e] + red[2][e] + red[3][e];
  }
}

// ---------------------------------------------------------------- elementwise
__device__ __forceinline__ float gelu_t(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}
__device__ __forceinline__ float gelu_t_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  const float t = tanhf(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
}

__global__ void __launch_bounds__(256) gelu_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    load8(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_t(v[j]);
    store8(y + i * 8, v);
  }
}

__global__ void __launch_bounds__(256) gelu_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                       bf16* __restrict__ dx, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8], g[8];
    load8(x + i * 8, v);
    load8(dy + i * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = g[j] * gelu_t_grad(v[j]);
    store8(dx + i * 8, v);
  }
}

// SwiGLU on a fused [N, 2F] projection: y = silu(a) * b, a = cols [0,F), b = cols [F,2F)
__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const bf16* __restrict__ ab, bf16* __restrict__ y, int64_t N,
                                                         int F) {
  const int64_t n8 = N * (F / 8);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / (F / 8);
    const int c = (int)(i % (F / 8)) * 8;
    float av[8], bv[8], o[8];
    load8(ab + row * 2 * F + c, av);
    load8(ab + row * 2 * F + F + c, bv);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = av[j] / (1.f + __expf(-av[j])) * bv[j];
    store8(y + row * F + c, o);
  }
}

__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ ab,
                                                         bf16* __restrict__ dab, int64_t N, int F) {
  const int64_t n8 = N * (F / 8);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / (F / 8);
    const int c = (int)(i % (F / 8)) * 8;
    float av[8], bv[8], g[8], da[8], db[8];
    load8(ab + row * 2 * F + c, av);
    load8(ab + row * 2 * F + F + c, bv);
    load8(dy + row * F + c, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = 1.f / (1.f + __expf(-av[j]));
      const float si = av[j] * sg;
      db[j] = g[j] * si;
      da[j] = g[j] * bv[j] * sg * (1.f + av[j] * (1.f - sg));
    }
    store8(dab + row * 2 * F + c, da);
    store8(dab + row * 2 * F + F + c, db);
  }
}

// Rotary embedding (rotate-half convention) in place on [B, S, heads, D] rows with
// token stride `ss` and batch stride `sb`; cos/sin tables [S, D/2] fp32.
// sign = +1 forward, -1 backward (rotation by -theta).
__global__ void __launch_bounds__(256) rope_kernel(bf16* __restrict__ x, const float* __restrict__ cs,
                                                   const float* __restrict__ sn, int B, int S, int heads, int D,
                                                   int64_t sb, int64_t ss, float sign) {
  const int half = D / 2;
  const int64_t total = (int64_t)B * S * heads * (half / 4);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(i % (half / 4)) * 4;
    int64_t r = i / (half / 4);
    const int h = r % heads;
    r /= heads;
    const int s = r % S;
    const int b = (int)(r / S);
    bf16* p = x + (int64_t)b * sb + (int64_t)s * ss + (int64_t)h * D;
    const bf16x4 x1 = *reinterpret_cast<const bf16x4*>(p + c4);
    const bf16x4 x2 = *reinterpret_cast<const bf16x4*>(p + half + c4);
    const float4 cv = *reinterpret_cast<const float4*>(cs + (int64_t)s * half + c4);
    const float4 sv = *reinterpret_cast<const float4*>(sn + (int64_t)s * half + c4);
    const float c[4] = {cv.x, cv.y, cv.z, cv.w}, sn4[4] = {sv.x * sign, sv.y * sign, sv.z * sign, sv.w * sign};
    bf16x4 o1, o2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = bf2f(x1[j]), bb = bf2f(x2[j]);
      o1[j] = f2bf(a * c[j] - bb * sn4[j]);
      o2[j] = f2bf(bb * c[j] + a * sn4[j]);
    }
    *reinterpret_cast<bf16x4*>(p + c4) = o1;
    *reinterpret_cast<bf16x4*>(p + half + c4) = o2;
  }
}

// Fused softmax cross-entropy: one workgroup per row; writes loss[row] and
// d(loss)/d(logits) * grad_scale into `dlogits` (may alias `logits`: in place).
// Rows with target == ignore_index get zero loss / gradient.
// NT threads per row: 1024 for the Llama-3 vocabulary -- 256-thread rows ran 8 workgroups per CU, 2048
// rows (512 MB) in flight, so the second pass's re-read of a row missed the 256 MB Infinity Cache and
// went back to HBM (6.3 GB of traffic per 8192-token step, 1.17 ms); 1024-thread rows keep ~512 rows
// (128 MB) in flight.
template <int NT>
__global__ void __launch_bounds__(NT) cross_entropy_kernel(const bf16* logits, bf16* dlogits,
                                                            const int64_t* __restrict__ target,
                                                            float* __restrict__ loss, int64_t V, float grad_scale,
                                                            int64_t ignore_index) {
  const int64_t row = blockIdx.x;
  const bf16* x = logits + row * V;
  bf16* dx = dlogits + row * V;
  const int64_t t = target[row];
  constexpr int NW = NT / 64;
  __shared__ float sm[NW], ss[NW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool vec = (V % 8) == 0;
  // pass 1: online max / sum-exp
  float m = -INFINITY, s = 0.f;
  // U chunks of 8 per thread in flight per iteration (one 16-B load each, all issued before any
  // use): with one load per iteration a CU held ~32 KB of reads in flight and the Llama-3 row
  // pass ran at ~3.5 TB/s
  constexpr int U = 4;
  if (vec) {
    for (int64_t c0 = (int64_t)threadIdx.x * 8; c0 < V; c0 += NT * 8 * U) {
      bf16x8 r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t c = c0 + (int64_t)u * NT * 8;
        if (c < V) r[u] = *reinterpret_cast<const bf16x8*>(x + c);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t c = c0 + (int64_t)u * NT * 8;
        if (c < V) {
          float mm = bf2f(r[u][0]);
#pragma unroll
          for (int j = 1; j < 8; ++j) mm = fmaxf(mm, bf2f(r[u][j]));
          const float mn = fmaxf(m, mm);
          s = s * __expf(m - mn);
#pragma unroll
          for (int j = 0; j < 8; ++j) s += __expf(bf2f(r[u][j]) - mn);
          m = mn;
        }
      }
    }
  } else {
    for (int64_t c = threadIdx.x; c < V; c += NT) {
      const float v = bf2f(x[c]);
      const float mn = fmaxf(m, v);
      s = s * __expf(m - mn) + __expf(v - mn);
      m = mn;
    }
  }
  // combine (m, s) across the wave, then across waves
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float mo = __shfl_xor(m, off, kWave), so = __shfl_xor(s, off, kWave);
    const float mn = fmaxf(m, mo);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (mo == -INFINITY ? 0.f : so * __expf(mo - mn));
    m = mn;
  }
  if (lane == 0) {
    sm[wave] = m;
    ss[wave] = s;
  }
  __syncthreads();
  float M = sm[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) M = fmaxf(M, sm[w]);
  float Ssum = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) Ssum += sm[w] == -INFINITY ? 0.f : ss[w] * __expf(sm[w] - M);
  const float lse = M + __logf(Ssum);
  const bool ignore = t == ignore_index || t < 0 || t >= V;
  const float xt = ignore ? 0.f : bf2f(x[ignore ? 0 : t]);
  __syncthreads();  // everyone has read x[t] before it may be overwritten (in place)
  if (threadIdx.x == 0) loss[row] = ignore ? 0.f : lse - xt;
  const float gs = ignore ? 0.f : grad_scale;
  // pass 2: gradient softmax - onehot
  if (vec) {
    for (int64_t c0 = (int64_t)threadIdx.x * 8; c0 < V; c0 += NT * 8 * U) {
      bf16x8 r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t c = c0 + (int64_t)u * NT * 8;
        if (c < V) r[u] = *reinterpret_cast<const bf16x8*>(x + c);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t c = c0 + (int64_t)u * NT * 8;
        if (c < V) {
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (__expf(bf2f(r[u][j]) - lse) - (c + j == t ? 1.f : 0.f)) * gs;
          store8(dx + c, v);
        }
      }
    }
  } else {
    for (int64_t c = threadIdx.x; c < V; c += NT) {
      const float v = bf2f(x[c]);
      dx[c] = f2bf((__expf(v - lse) - (c == t ? 1.f : 0.f)) * gs);
    }
  }
}

// Opaque to the compiler: the row stays packed bf16 (4 VGPRs per chunk) between
// passes instead of being kept converted to fp32 (8 per chunk), which would cut
// occupancy to one wave per SIMD; re-widening is one shift per value.
template <int CH>
__device__ __forceinline__ void keep_packed(bf16x8 (&r)[CH]) {
  typedef int i4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    i4 w = __builtin_bit_cast(i4, r[k]);
    asm volatile("" : "+v"(w));
    r[k] = __builtin_bit_cast(bf16x8, w);
  }
}

// Same op with the row held in registers between the two passes, so it is
// read from HBM once (the two-pass kernel above re-reads its 100 KB GPT-2 row,
// mostly from the Infinity Cache): NT threads x CH chunks of 8 bf16 cover up
// to NT * 8 * CH logits; V % 8 == 0.  (GPT-2 vocabulary; a Llama-3 row would
// need 1024 threads x 16 chunks, over the 128 VGPRs such a block allows.)
template <int NT, int CH>
__global__ void __launch_bounds__(NT) cross_entropy_rows_kernel(const bf16* logits, bf16* dlogits,
                                                                const int64_t* __restrict__ target,
                                                                float* __restrict__ loss, int64_t V,
                                                                float grad_scale, int64_t ignore_index) {
  constexpr int NW = NT / 64;
  const int64_t row = blockIdx.x;
  const bf16* x = logits + row * V;
  bf16* dx = dlogits + row * V;
  const int64_t t = target[row];
  __shared__ float sm[NW], ss[NW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  bf16x8 r[CH];
#pragma unroll
  for (int k = 0; k < CH; ++k) {  // every load in flight before any use
    const int64_t c = ((int64_t)k * NT + threadIdx.x) * 8;
    if (c < V) r[k] = *reinterpret_cast<const bf16x8*>(x + c);
  }
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int64_t c = ((int64_t)k * NT + threadIdx.x) * 8;
    if (c < V)
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, bf2f(r[k][j]));
  }
  m = wave_max(m);
  keep_packed<CH>(r);
  if (lane == 0) sm[wave] = m;
  __syncthreads();
  float M = sm[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) M = fmaxf(M, sm[w]);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int64_t c = ((int64_t)k * NT + threadIdx.x) * 8;
    if (c < V)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(bf2f(r[k][j]) - M);
  }
  s = wave_sum(s);
  keep_packed<CH>(r);
  if (lane == 0) ss[wave] = s;
  __syncthreads();
  float Ssum = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) Ssum += ss[w];
  const float lse = M + __logf(Ssum);
  const bool ignore = t == ignore_index || t < 0 || t >= V;
  const float xt = ignore ? 0.f : bf2f(x[ignore ? 0 : t]);
  if (threadIdx.x == 0) loss[row] = ignore ? 0.f : lse - xt;
  __syncthreads();  // x[t] read by thread 0 before it may be overwritten (in place)
  const float gs = ignore ? 0.f : grad_scale;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int64_t c = ((int64_t)k * NT + threadIdx.x) * 8;
    if (c < V) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__expf(bf2f(r[k][j]) - lse) - (c + j == t ? 1.f : 0.f)) * gs;
      store8(dx + c, v);
    }
  }
}

static inline int egrid(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}


// ---------------------------------------------------------------- embedding backward
// dW[id] += sum of the rows of dy whose token is id -- deterministic, no atomics: the ids come
// sorted (stable) with their source rows; the workgroup of position t works only when t starts
// a run of equal ids and sums that run's rows in fp32, in source order, then adds the sum into
// the bf16 row of `out` (read-modify-write of one row: `out` may already hold another use's
// gradient, e.g. the tied LM head's, which is then accumulated rather than summed by autograd).
// Reference: the token/position embeddings of the GPT-2 configs (SURVEY.md §2.5 N07 models).
__global__ void __launch_bounds__(128) embedding_bwd_kernel(const int64_t* __restrict__ sid,
                                                           const int64_t* __restrict__ perm,
                                                           const bf16* __restrict__ dy, bf16* __restrict__ out,
                                                           int T, int C, int64_t ldo, int64_t V) {
  const int t = blockIdx.x;
  const int64_t id = sid[t];
  if ((t > 0 && sid[t - 1] == id) || id < 0 || id >= V) return;
  int end = t + 1;
  while (end < T && sid[end] == id) ++end;
  for (int c = threadIdx.x * 8; c < C; c += blockDim.x * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = t; r < end; ++r) {
      float f[8];
      load8(dy + perm[r] * (int64_t)C + c, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    bf16* o = out + id * ldo + c;
    float f[8];
    load8(o, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] += acc[j];
    store8(o, f);
  }
}

// ---------------------------------------------------------------- CE mean
// loss = sum(rows) / max(1, #(target != ignore)) and that divisor, in ONE single-workgroup launch (the
// torch-op form -- compare, sum, clamp, casts, sum, divide -- was 7-9 launches, ~40 us per GPT-2 step).
// Fixed reduction order (lane stride, then waves 0..15): the same bits every call.
__global__ void __launch_bounds__(1024) ce_mean_kernel(const float* __restrict__ rows,
                                                       const int64_t* __restrict__ target, int64_t N,
                                                       int64_t ignore_index, float* __restrict__ loss,
                                                       float* __restrict__ count) {
  __shared__ float ps[16], pc[16];
  float s = 0.f, c = 0.f;
  for (int64_t i = threadIdx.x; i < N; i += 1024) {
    s += rows[i];
    c += target[i] != ignore_index ? 1.f : 0.f;
  }
  s = wave_sum(s);
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) {
    ps[threadIdx.x >> 6] = s;
    pc[threadIdx.x >> 6] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float S = 0.f, C = 0.f;
    for (int w = 0; w < 16; ++w) {
      S += ps[w];
      C += pc[w];
    }
    C = fmaxf(C, 1.f);
    *loss = S / C;
    *count = C;
  }
}

}  // namespace dta

using namespace dta;

hipError_t dta_ce_mean(const float* rows, const int64_t* target, int64_t N, int64_t ignore_index, float* loss,
                       float* count, hipStream_t st) {
  if (N < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ce_mean_kernel, dim3(1), dim3(1024), 0, st, rows, target, N, ignore_index, loss, count);
  return hipGetLastError();
}

template <bool RMS>
static hipError_t norm_fwd_nv(int nv, const bf16* x, const bf16* w, const bf16* b, bf16* y, float* mean, float* rstd,
                              int64_t N, int C, float eps, const bf16* res, bf16* xsum, hipStream_t st) {
  dim3 grid((unsigned)((N + 3) / 4)), blk(256);
  switch (nv) {
    case 1: hipLaunchKernelGGL((norm_fwd_kernel<1, RMS>), grid, blk, 0, st, x, w, b, y, mean, rstd, N, C, eps, res, xsum); break;
    case 2: hipLaunchKernelGGL((norm_fwd_kernel<2, RMS>), grid, blk, 0, st, x, w, b, y, mean, rstd, N, C, eps, res, xsum); break;
    case 4: hipLaunchKernelGGL((norm_fwd_kernel<4, RMS>), grid, blk, 0, st, x, w, b, y, mean, rstd, N, C, eps, res, xsum); break;
    case 8: hipLaunchKernelGGL((norm_fwd_kernel<8, RMS>), grid, blk, 0, st, x, w, b, y, mean, rstd, N, C, eps, res, xsum); break;
    case 16: hipLaunchKernelGGL((norm_fwd_kernel<16, RMS>), grid, blk, 0, st, x, w, b, y, mean, rstd, N, C, eps, res, xsum); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

static int nv_for(int C) {
  const int v = (C + 511) / 512;
  if (v <= 1) return 1;
  if (v <= 2) return 2;
  if (v <= 4) return 4;
  if (v <= 8) return 8;
  if (v <= 16) return 16;
  return -1;
}

hipError_t dta_norm_fwd(bool rms, const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                        int64_t N, int C, float eps, const void* res, void* xsum, hipStream_t st) {
  const int nv = nv_for(C);
  if (nv < 0 || C % 8) return hipErrorInvalidValue;
  auto X = reinterpret_cast<const bf16*>(x);
  auto W = reinterpret_cast<const bf16*>(w);
  auto Bv = reinterpret_cast<const bf16*>(b);
  auto Y = reinterpret_cast<bf16*>(y);
  auto R = reinterpret_cast<const bf16*>(res);
  auto XS = reinterpret_cast<bf16*>(xsum);
  return rms ? norm_fwd_nv<true>(nv, X, W, Bv, Y, mean, rstd, N, C, eps, R, XS, st)
             : norm_fwd_nv<false>(nv, X, W, Bv, Y, mean, rstd, N, C, eps, R, XS, st);
}

template <bool RMS>
static hipError_t norm_bwd_nv(int nv, const bf16* dy, const bf16* x, const bf16* w, const float* mean,
                              const float* rstd, bf16* dx, float* dwp, float* dbp, int64_t N, int C, int rpb,
                              const bf16* dres, hipStream_t st) {
  dim3 grid((unsigned)((N + rpb - 1) / rpb)), blk(256);
  if (C % 2048 == 0 && C <= 8192) {  // wide rows: a workgroup per row (norm_bwd_wide_kernel)
#define NW_(V) \
  hipLaunchKernelGGL((norm_bwd_wide_kernel<V, RMS>), grid, blk, 0, st, dy, x, w, mean, rstd, dx, dwp, dbp, N, C, rpb, dres)
    switch (C / 2048) {
      case 1: NW_(1); break;
      case 2: NW_(2); break;
      case 3: NW_(3); break;
      default: NW_(4); break;
    }
#undef NW_
    return hipGetLastError();
  }
#define NB(V) \
  hipLaunchKernelGGL((norm_bwd_kernel<V, RMS>), grid, blk, 0, st, dy, x, w, mean, rstd, dx, dwp, dbp, N, C, rpb, dres)
  switch (nv) {
    case 1: NB(1); break;
    case 2: NB(2); break;
    case 4: NB(4); break;
    case 8: NB(8); break;
    case 16: NB(16); break;
    default: return hipErrorInvalidValue;
  }
#undef NB
  return hipGetLastError();
}

// dw/db partial workspace: [nblk][C] fp32 each, nblk = ceil(N / rows_per_block)
hipError_t dta_norm_bwd(bool rms, const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                        void* dx, float* dw_part, float* db_part, void* dw, void* db, int64_t N, int C,
                        int rows_per_block, int grads_f32, const void* dres, hipStream_t st) {
  const int nv = nv_for(C);
  if (nv < 0 || C % 8) return hipErrorInvalidValue;
  auto r = rms ? norm_bwd_nv<true>(nv, (const bf16*)dy, (const bf16*)x, (const bf16*)w, mean, rstd, (bf16*)dx,
                                   dw_part, db_part, N, C, rows_per_block, (const bf16*)dres, st)
               : norm_bwd_nv<false>(nv, (const bf16*)dy, (const bf16*)x, (const bf16*)w, mean, rstd, (bf16*)dx,
                                    dw_part, db_part, N, C, rows_per_block, (const bf16*)dres, st);
  if (r != hipSuccess) return r;
  const int nblk = (int)((N + rows_per_block - 1) / rows_per_block);
  const int nb = (C + 31) / 32;
  bf16* w16 = grads_f32 ? nullptr : (bf16*)dw;
  float* w32 = grads_f32 ? (float*)dw : nullptr;
  bf16* b16 = grads_f32 ? nullptr : (bf16*)db;
  float* b32 = grads_f32 ? (float*)db : nullptr;
  if (!dw && !db) return hipSuccess;  // deferred: the caller finishes the partials (dta_colsum_batch)
  hipLaunchKernelGGL(colsum_kernel, dim3(rms ? nb : 2 * nb), dim3(256), 0, st, dw_part, db_part, nblk, C, w16, w32, b16,
                     b32);
  return hipGetLastError();
}

int dta_colsum_batch_max() { return ColsumJobs::kMax; }

// out_j[c] = sum_r part_j[r][c] for n <= kMax jobs in one launch (bf16 outputs)
hipError_t dta_colsum_batch(int n, const float* const* part, const int* nrows, const int* C, void* const* out,
                            hipStream_t st) {
  if (n < 1 || n > ColsumJobs::kMax) return hipErrorInvalidValue;
  ColsumJobs jobs{};
  jobs.n = n;
  int total = 0;
  for (int j = 0; j < n; ++j) {
    jobs.start[j] = total;
    jobs.part[j] = part[j];
    jobs.nrows[j] = nrows[j];
    jobs.C[j] = C[j];
    jobs.out[j] = static_cast<bf16*>(out[j]);
    total += (C[j] + 31) / 32;
  }
  jobs.start[n] = total;
  hipLaunchKernelGGL(colsum_batch_kernel, dim3((unsigned)total), dim3(256), 0, st, jobs);
  return hipGetLastError();
}

// out[c] = sum_r part[r][c] (fp32 [nrows][C] partials -> bf16 / f32)
hipError_t dta_colsum_partials(const float* part, int nrows, int C, void* out, int out_f32, hipStream_t st) {
  hipLaunchKernelGGL(colsum_kernel, dim3((C + 31) / 32), dim3(256), 0, st, part, static_cast<const float*>(nullptr),
                     nrows, C, out_f32 ? nullptr : (bf16*)out, out_f32 ? (float*)out : nullptr,
                     static_cast<bf16*>(nullptr), static_cast<float*>(nullptr));
  return hipGetLastError();
}

hipError_t dta_bias_grad(const void* dy, int64_t N, int C, float* part, int nsplit, void* out, int out_f32,
                         hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const int rps = (int)((N + nsplit - 1) / nsplit);
  hipLaunchKernelGGL(colsum_bf16_partial_kernel, dim3((C + 511) / 512, nsplit), dim3(256), 0, st, (const bf16*)dy, N,
                     C, rps, part);
  hipLaunchKernelGGL(colsum_kernel, dim3((C + 31) / 32), dim3(256), 0, st, part, static_cast<const float*>(nullptr),
                     nsplit, C, out_f32 ? nullptr : (bf16*)out, out_f32 ? (float*)out : nullptr,
                     static_cast<bf16*>(nullptr), static_cast<float*>(nullptr));
  return hipGetLastError();
}

hipError_t dta_gelu_fwd(const void* x, void* y, int64_t n, hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(egrid(n / 8)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, n / 8);
  return hipGetLastError();
}
hipError_t dta_gelu_bwd(const void* dy, const void* x, void* dx, int64_t n, hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(egrid(n / 8)), dim3(256), 0, st, (const bf16*)dy, (const bf16*)x,
                     (bf16*)dx, n / 8);
  return hipGetLastError();
}
hipError_t dta_swiglu_fwd(const void* ab, void* y, int64_t N, int F, hipStream_t st) {
  if (F % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(egrid(N * F / 8)), dim3(256), 0, st, (const bf16*)ab, (bf16*)y, N, F);
  return hipGetLastError();
}
hipError_t dta_swiglu_bwd(const void* dy, const void* ab, void* dab, int64_t N, int F, hipStream_t st) {
  if (F % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(egrid(N * F / 8)), dim3(256), 0, st, (const bf16*)dy, (const bf16*)ab,
                     (bf16*)dab, N, F);
  return hipGetLastError();
}
hipError_t dta_rope(void* x, const float* cs, const float* sn, int B, int S, int heads, int D, int64_t sb, int64_t ss,
                    float sign, hipStream_t st) {
  if (D % 8) return hipErrorInvalidValue;
  const int64_t total = (int64_t)B * S * heads * (D / 8);
  hipLaunchKernelGGL(rope_kernel, dim3(egrid(total)), dim3(256), 0, st, (bf16*)x, cs, sn, B, S, heads, D, sb, ss,
                     sign);
  return hipGetLastError();
}
hipError_t dta_cross_entropy(const void* logits, void* dlogits, const int64_t* target, float* loss, int64_t N,
                             int64_t V, float grad_scale, int64_t ignore_index, hipStream_t st) {
  const bf16* L = (const bf16*)logits;
  bf16* DL = (bf16*)dlogits;
  if (V % 8 == 0 && V <= 512 * 8 * 13) {  // GPT-2 (50304): 13 chunks of 8 per thread
    hipLaunchKernelGGL((cross_entropy_rows_kernel<512, 13>), dim3((unsigned)N), dim3(512), 0, st, L, DL, target, loss,
                       V, grad_scale, ignore_index);
  } else {  // larger vocabularies (Llama-3: 128256) stream the row twice
    hipLaunchKernelGGL(cross_entropy_kernel<1024>, dim3((unsigned)N), dim3(1024), 0, st, L, DL, target, loss, V, grad_scale,
                       ignore_index);
  }
  return hipGetLastError();
}

hipError_t dta_embedding_bwd(const int64_t* sid, const int64_t* perm, const void* dy, void* out, int T, int C,
                             int64_t ldo, int64_t V, hipStream_t st) {
  if (C % 8 || ldo % 8 || T <= 0) return T <= 0 ? hipSuccess : hipErrorInvalidValue;
  hipLaunchKernelGGL(embedding_bwd_kernel, dim3(T), dim3(128), 0, st, sid, perm, (const bf16*)dy, (bf16*)out, T, C,
                     ldo, V);
  return hipGetLastError();
}
