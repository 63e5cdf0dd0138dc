// Weight-gradient GEMM for gfx950:  C[M, N] = A^T . B  with A [K, M] and
// B [K, N] both row-major (K = tokens).  This is dW = dY^T . X of every
// Linear layer (the "dW" GEMM of §7.1 gemm.hip).
//
// Why a hand-written kernel: at transformer shapes the weight gradient has a
// small output (768 x 3072 for GPT-2 small = 144 tiles of 128 x 128) and a
// long reduction (K = B*S = 8192 tokens), so a library GEMM that tiles only the
// output under-fills 256 CUs (measured: hipBLASLt 190-480 TF/s on the four
// GPT-2 shapes).  Here the reduction is split over a third grid dimension
// (split-K) so the launch fills the CUs, and the fp32 slabs are summed by a
// small vectorised reduce kernel into the bf16 gradient.
//
// Both operands have the reduction index as their ROW index, so both MFMA
// fragments are read column-wise: tiles are staged row-major in LDS (256-B rows,
// 16-B chunks XOR-swizzled so row reads and transposed reads are bank-conflict
// free, cdna_hip_programming.md T10 layout (b)) and fragments come from
// ds_read_b64_tr_b16.  Workgroup = 4 waves (2 x 2), 128 x 128 output tile, each
// wave 64 x 64 = 2 x 2 v_mfma_f32_32x32x16_bf16 tiles.
//
// Two kernels: gemm_tn_gd_kernel (default; LDS-DMA staging into a 4-deep ring
// of 32-token stages, any split) and gemm_tn_kernel (register staging, 64-token
// stages, double-buffered; kept for A/B runs).  GPT-2 shapes, one MI355X:
// qkv 52.2 -> 46.5 us, proj 28.9 -> 23.8, fc 75.9 -> 58.3, fc2 76.6 -> 59.9.
#include "common.h"

namespace dta {

constexpr int kGtBM = 128, kGtBN = 128, kGtBK = 64;
constexpr int kGtTileBytes = kGtBK * 256;  // one [64][128] bf16 tile

// byte offset of 16-byte chunk `ch` (0..15) of row `row` in a 256-B-row tile
__device__ __forceinline__ int gt_off(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ bf16x4 gt_tr4(const char* lds, int byte_off) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(lds + byte_off));
  return __builtin_bit_cast(bf16x4, v);
}

// MFMA operand fragment X^T for k-step s and 32 columns starting at c0 of the
// [64 k][128 col] tile: lane l gets X[16s + 8(l>>5) + j][c0 + (l & 31)], j = 0..7.
__device__ __forceinline__ bf16x8 gt_frag(const char* tile, int s, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = 16 * s + 8 * (g >> 1) + (i >> 2);
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const int ch = col >> 3, sub = (col & 7) * 2;
  const bf16x4 lo = gt_tr4(tile, gt_off(row, ch) + sub);
  const bf16x4 hi = gt_tr4(tile, gt_off(row + 4, ch) + sub);
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

struct GemmTnArgs {
  const bf16* a;  // [K, M], row stride lda
  const bf16* b;  // [K, N], row stride ldb
  void* c;        // split == 1: bf16/f32 [M, N]; split > 1: f32 slabs [split][M][N]
  int64_t lda, ldb, ldc;
  int M, N, K, split, k_per_split;
  int tiles_m, tiles_n;
  int out_f32;
  // column sums of A (the bias gradient sum_k dY[k, m] of the same Linear) by
  // `cs_workers` extra workgroups of the same launch: f32 [cs_workers][M]
  // partials, summed by splitk_reduce_kernel (nullptr: off)
  float* colsum;
  int cs_workers, gemm_wgs;
};

// Extra workgroup of a gemm_tn launch: column sums of A over its share of the
// K rows.  The GEMM grid leaves most CUs' second workgroup slot idle at these
// shapes (e.g. 288 GEMM workgroups on 256 CUs x 2 slots), and these run there,
// so the bias gradient costs neither a separate pass nor GEMM-workgroup time.
__device__ void gemm_tn_colsum_worker(const GemmTnArgs& g, int w) {
  const int rows = (g.K + g.cs_workers - 1) / g.cs_workers;
  const int k0 = w * rows, k1 = min(g.K, k0 + rows);
  for (int c8 = threadIdx.x * 8; c8 < g.M; c8 += 256 * 8) {  // 8 columns per thread
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    int k = k0;
    for (; k + 8 <= k1; k += 8) {  // 8 rows in flight
      bf16x8 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const bf16x8*>(g.a + (int64_t)(k + u) * g.lda + c8);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[u][j]);
    }
    for (; k < k1; ++k) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(g.a + (int64_t)k * g.lda + c8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
    }
    float* out = g.colsum + (int64_t)w * g.M + c8;
    reinterpret_cast<float4*>(out)[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    reinterpret_cast<float4*>(out)[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
}

template <bool SLAB>
__global__ void __launch_bounds__(256) gemm_tn_kernel(GemmTnArgs g) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * kGtTileBytes];  // [buf][A|B][64][256 B]
  if ((int)blockIdx.x >= g.gemm_wgs) {  // column-sum workers (after every GEMM workgroup)
    gemm_tn_colsum_worker(g, blockIdx.x - g.gemm_wgs);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // bijective XCD remap: consecutive logical tiles (same split, neighbouring
  // output tiles -> shared A/B panels) land on the same XCD's L2
  const int nwg = g.gemm_wgs, orig = blockIdx.x;
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int tiles = g.tiles_m * g.tiles_n;
  const int sp = wg / tiles, t = wg % tiles;
  const int tm = t / g.tiles_n, tn = t % g.tiles_n;
  const int m0 = tm * kGtBM, n0 = tn * kGtBN;
  const int kbeg = sp * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int ntile = (kend - kbeg) / kGtBK;

  // staging: 4 chunks of A and 4 of B per thread per stage (chunk e: row e>>4, 16-B chunk e&15)
  bf16x8 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int e = tid + 256 * l, row = e >> 4, ch = e & 15;
      ra[l] = *reinterpret_cast<const bf16x8*>(g.a + (int64_t)(k0 + row) * g.lda + m0 + ch * 8);
      rb[l] = *reinterpret_cast<const bf16x8*>(g.b + (int64_t)(k0 + row) * g.ldb + n0 + ch * 8);
    }
  };
  auto lstore = [&](int buf) {
    char* ta = lds + buf * 2 * kGtTileBytes;
    char* tb = ta + kGtTileBytes;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int e = tid + 256 * l, row = e >> 4, ch = e & 15;
      *reinterpret_cast<bf16x8*>(ta + gt_off(row, ch)) = ra[l];
      *reinterpret_cast<bf16x8*>(tb + gt_off(row, ch)) = rb[l];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  if (ntile > 0) {
    gload(kbeg);
    lstore(0);
    __syncthreads();
  }
  for (int kt = 0; kt < ntile; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < ntile) gload(kbeg + (kt + 1) * kGtBK);
    const char* ta = lds + buf * 2 * kGtTileBytes;
    const char* tb = ta + kGtTileBytes;
#pragma unroll
    for (int s = 0; s < kGtBK / 16; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = gt_frag(ta, s, wm * 64 + 32 * i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = gt_frag(tb, s, wn * 64 + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32x32x16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < ntile) lstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: acc[i][j] rows m = m0 + wm*64 + 32i + mfma32_row(e), cols n = n0 + wn*64 + 32j + (lane & 31)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + 32 * j + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * 64 + 32 * i + mfma32_row(e, lane);
        if (SLAB) {
          static_cast<float*>(g.c)[((int64_t)sp * g.M + m) * g.N + n] = acc[i][j][e];
        } else if (g.out_f32) {
          static_cast<float*>(g.c)[(int64_t)m * g.ldc + n] = acc[i][j][e];
        } else {
          static_cast<bf16*>(g.c)[(int64_t)m * g.ldc + n] = f2bf(acc[i][j][e]);
        }
      }
    }
}

// ---------------------------------------------------------------------------
// LDS-DMA form (the default): split-K with a 4-deep ring of 32-token stages.
//
// What the measurements of gemm_tn_kernel said, and what changed:
//  * the register-staged form spends ~13 LDS cycles per ds_write_b128
//    wave-instruction (~415 LDS cycles per 64-token stage against 512 MFMA
//    cycles).  Here stages arrive by global_load_lds_dwordx4: one
//    wave-instruction writes 1 KiB (4 rows of the 256-B-row image) in 4 LDS
//    cycles; the XOR swizzle moves to the per-lane SOURCE address (the image is
//    lane-linear: row 4i + lane/16, physical chunk lane%16 holds logical chunk
//    (lane%16) ^ swz(row)); the 32 staging VGPRs are gone.
//  * one stage in flight left every stage waiting on L2/HBM latency (a stream-K
//    variant of the 2-buffer loop measured ~1.4 us per 64-token stage per CU).
//    Four 16-KiB buffers keep three stages in flight; the wait before each
//    barrier is a counted vmcnt (never 0 in the loop); 64 KiB per workgroup,
//    two workgroups per CU.
//  * stream-K (equal contiguous ranges of the (tile, k) space) lost: neighbour
//    workgroups then share a tile at DIFFERENT k, so nothing is reused from L2.
//    Split-K keeps neighbours on one k-range of neighbouring tiles (shared A/B
//    panels on one XCD); splits need not divide K (floor ranges), so the split
//    can be chosen to fill the 512 workgroup slots.
// ---------------------------------------------------------------------------
constexpr int kGdBK = 32, kGdStage = 2 * kGdBK * 256, kGdBufs = 4;  // stage = A [32][256 B] + B [32][256 B]

struct GemmGdArgs {
  const bf16* a;
  const bf16* b;
  void* c;  // split == 1: bf16/f32 [M, ldc]; split > 1: f32 slabs [split][M][N]
  int64_t lda, ldb, ldc;
  int M, N, K, split, tiles_n, tiles, kt_total, out_f32;
  float* colsum;
  int cs_workers, gemm_wgs;
};

// wait until at most 4 * `stages` of this wave's LDS-DMA loads are outstanding
__device__ __forceinline__ void vm_wait(int stages) {
  if (stages >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (stages == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool SLAB>
__global__ void __launch_bounds__(256, 2) gemm_tn_gd_kernel(GemmGdArgs g) {
  __shared__ __attribute__((aligned(1024))) char lds[kGdBufs * kGdStage];
  if ((int)blockIdx.x >= g.gemm_wgs) {
    GemmTnArgs t{};
    t.a = g.a;
    t.lda = g.lda;
    t.M = g.M;
    t.K = g.K;
    t.colsum = g.colsum;
    t.cs_workers = g.cs_workers;
    gemm_tn_colsum_worker(t, blockIdx.x - g.gemm_wgs);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = g.gemm_wgs, orig = blockIdx.x;
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int sp = wg / g.tiles, t = wg - sp * g.tiles;
  const int tm = t / g.tiles_n, tn = t - tm * g.tiles_n;
  const int m0 = tm * kGtBM, n0 = tn * kGtBN;
  const int kt0 = (int)((int64_t)sp * g.kt_total / g.split), kt1 = (int)((int64_t)(sp + 1) * g.kt_total / g.split);
  const int n = kt1 - kt0;

  // per-lane source pieces: wave w issues instructions i = 2w, 2w+1 of each operand (rows 4i .. 4i+3)
  const int lrow = lane >> 4, pc = lane & 15;
  const bf16* srcA[2];
  const bf16* srcB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = wave * 2 + j, row = 4 * i + lrow;
    const int ch = pc ^ ((lrow << 2) | (i & 3));  // gt_off's swizzle at row 4i + lrow
    srcA[j] = g.a + (int64_t)(kt0 * kGdBK + row) * g.lda + m0 + ch * 8;
    srcB[j] = g.b + (int64_t)(kt0 * kGdBK + row) * g.ldb + n0 + ch * 8;
  }
  auto issue = [&](int stage) {  // stage index relative to kt0
    char* ta = lds + (stage & (kGdBufs - 1)) * kGdStage;
    char* tb = ta + kGdBK * 256;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = wave * 2 + j;
      glds16(srcA[j] + (int64_t)stage * kGdBK * g.lda, ta + i * 1024);
      glds16(srcB[j] + (int64_t)stage * kGdBK * g.ldb, tb + i * 1024);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int pre = min(n, kGdBufs - 1);
  for (int s = 0; s < pre; ++s) issue(s);
  vm_wait(pre - 1);  // stage 0 landed
  __syncthreads();
  for (int kt = 0; kt < n; ++kt) {
    // the buffer of stage kt+3 was last read in iteration kt-1, before its barrier
    if (kt + kGdBufs - 1 < n) issue(kt + kGdBufs - 1);
    const char* ta = lds + (kt & (kGdBufs - 1)) * kGdStage;
    const char* tb = ta + kGdBK * 256;
#pragma unroll
    for (int s = 0; s < kGdBK / 16; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = gt_frag(ta, s, wm * 64 + 32 * i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = gt_frag(tb, s, wn * 64 + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32x32x16(af[i], bfr[j], acc[i][j]);
    }
    // stage kt+1 landed (this wave's part; the barrier makes it every wave's):
    // stages issued after it = min(n - 1, kt + 3) - (kt + 1)
    vm_wait(min(n - 1, kt + kGdBufs - 1) - (kt + 1));
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nn = n0 + wn * 64 + 32 * j + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * 64 + 32 * i + mfma32_row(e, lane);
        if (SLAB) {
          static_cast<float*>(g.c)[((int64_t)sp * g.M + m) * g.N + nn] = acc[i][j][e];
        } else if (g.out_f32) {
          static_cast<float*>(g.c)[(int64_t)m * g.ldc + nn] = acc[i][j][e];
        } else {
          static_cast<bf16*>(g.c)[(int64_t)m * g.ldc + nn] = f2bf(acc[i][j][e]);
        }
      }
    }
}

// out[M, N] = sum_s slab[s][M][N]   (bf16 or f32 out, 4 elements per thread);
// blocks past the matrix finish the bias gradient from the column-sum
// partials in the same launch: cout[m] = sum_w cs[w][m] (colsum_block)
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ slab, int split, int64_t mn,
                                                            void* out, int out_f32, const float* __restrict__ cs,
                                                            int M, void* cout, int cout_f32, int ncs) {
  const int64_t mblocks = (mn / 4 + 255) / 256;
  if ((int64_t)blockIdx.x >= mblocks) {
    const int c0 = (int)((int64_t)blockIdx.x - mblocks) * 32;
    colsum_block(cs, ncs, M, c0, cout_f32 ? nullptr : static_cast<bf16*>(cout),
                 cout_f32 ? static_cast<float*>(cout) : nullptr);
    return;
  }
  const int64_t i4 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i4 * 4 >= mn) return;
  float4 acc = reinterpret_cast<const float4*>(slab)[i4];
  for (int s = 1; s < split; ++s) {
    const float4 v = reinterpret_cast<const float4*>(slab + (int64_t)s * mn)[i4];
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  if (out_f32) {
    reinterpret_cast<float4*>(out)[i4] = acc;
  } else {
    bf16x4 o = {f2bf(acc.x), f2bf(acc.y), f2bf(acc.z), f2bf(acc.w)};
    reinterpret_cast<bf16x4*>(out)[i4] = o;
  }
}

}  // namespace dta

using namespace dta;

// Split until the launch has >= 256 workgroups (one per CU; measured best on the
// GPT-2 shapes), each split >= 4 stages deep.
int dta_gemm_tn_split(int M, int N, int K) {
  if (M % kGtBM || N % kGtBN || K % kGtBK) return 0;
  const int tiles = (M / kGtBM) * (N / kGtBN);
  int split = 1;
  while (tiles * split < 256 && K / (split * 2) >= 4 * kGtBK && (K / kGtBK) % (split * 2) == 0) split *= 2;
  return split;
}

// c: [M, N] (bf16 or f32, row stride ldc); slab: f32 [split * M * N] when split > 1
// colsum (optional): f32 [dta_gemm_tn_cs_workers(K)][M] scratch; cout: the bias gradient [M] (bf16 / f32 as out_f32)
// 64 rows per worker: 8 row loads in flight per thread, and enough workers to
// fill the CU slots the GEMM grid leaves idle (partials summed by colsum_kernel)
int dta_gemm_tn_cs_workers(int K) { return (K + 63) / 64; }
hipError_t dta_colsum_partials(const float* part, int nrows, int C, void* out, int out_f32, hipStream_t st);

hipError_t dta_gemm_tn(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, int M, int N,
                       int K, int split, float* slab, int out_f32, float* colsum, void* cout, hipStream_t st) {
  if (M % kGtBM || N % kGtBN || K % kGtBK || split < 1 || (K / kGtBK) % split) return hipErrorInvalidValue;
  GemmTnArgs g{};
  g.a = static_cast<const bf16*>(a);
  g.b = static_cast<const bf16*>(b);
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.split = split;
  g.k_per_split = K / split;
  g.tiles_m = M / kGtBM;
  g.tiles_n = N / kGtBN;
  g.out_f32 = out_f32;
  g.colsum = cout ? colsum : nullptr;
  if (cout && !colsum) return hipErrorInvalidValue;
  if (cout && M % 8) return hipErrorInvalidValue;
  g.gemm_wgs = g.tiles_m * g.tiles_n * split;
  g.cs_workers = cout ? dta_gemm_tn_cs_workers(K) : 0;
  const int grid = g.gemm_wgs + g.cs_workers;
  if (split == 1) {
    g.c = c;
    hipLaunchKernelGGL(gemm_tn_kernel<false>, dim3(grid), dim3(256), 0, st, g);
  } else {
    if (ldc != N) return hipErrorInvalidValue;
    g.c = slab;
    hipLaunchKernelGGL(gemm_tn_kernel<true>, dim3(grid), dim3(256), 0, st, g);
    const int64_t mn = (int64_t)M * N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((mn / 4 + 255) / 256)), dim3(256), 0, st, slab, split, mn,
                       c, out_f32, static_cast<const float*>(nullptr), 0, static_cast<void*>(nullptr), 0, 0);
  }
  if (cout) DTA_HIP_CHECK(dta_colsum_partials(colsum, g.cs_workers, M, cout, out_f32, st));
  return hipGetLastError();
}

// LDS-DMA split-K form.  split = 0: pick it (dta_gemm_tn_gd_split).  slab: f32
// [split * M * N] when split > 1.
static int gd_wgs(int tiles, int split) { return tiles * split; }

// Fill the 512 workgroup slots (256 CUs x 2): minimise rounds x stages per
// workgroup, each split >= 8 stages (256 tokens) deep, plus the slab round trip.
int dta_gemm_tn_gd_split(int M, int N, int K) {
  if (M % kGtBM || N % kGtBN || K % kGdBK) return 0;
  const int tiles = (M / kGtBM) * (N / kGtBN), kt = K / kGdBK;
  int best = 1;
  double best_cost = 1e30;
  for (int sp = 1; sp <= 64 && kt / sp >= 8; ++sp) {
    const int rounds = (gd_wgs(tiles, sp) + 511) / 512;
    const double stages = (double)rounds * ((kt + sp - 1) / sp);
    // slab: split x M x N f32 written and read; ~1 stage-time per 2 MB per round of 512 (measured scale)
    const double slab = sp > 1 ? (double)sp * M * N * 8.0 / (2.0 * 1024 * 1024) : 0.0;
    const double cost = stages + slab;
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = sp;
    }
  }
  return best;
}

hipError_t dta_gemm_tn_gd(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, int M, int N,
                          int K, int split, float* slab, int out_f32, float* colsum, void* cout, hipStream_t st) {
  if (M % kGtBM || N % kGtBN || K % kGdBK || split < 1 || split > K / kGdBK) return hipErrorInvalidValue;
  if (cout && (!colsum || M % 8)) return hipErrorInvalidValue;
  GemmGdArgs g{};
  g.a = static_cast<const bf16*>(a);
  g.b = static_cast<const bf16*>(b);
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.split = split;
  g.tiles_n = N / kGtBN;
  g.tiles = (M / kGtBM) * g.tiles_n;
  g.kt_total = K / kGdBK;
  g.out_f32 = out_f32;
  g.colsum = cout ? colsum : nullptr;
  g.gemm_wgs = gd_wgs(g.tiles, split);
  g.cs_workers = cout ? dta_gemm_tn_cs_workers(K) : 0;
  const int grid = g.gemm_wgs + g.cs_workers;
  if (split == 1) {
    g.c = c;
    hipLaunchKernelGGL(gemm_tn_gd_kernel<false>, dim3(grid), dim3(256), 0, st, g);
  } else {
    if (ldc != N || !slab) return hipErrorInvalidValue;
    g.c = slab;
    hipLaunchKernelGGL(gemm_tn_gd_kernel<true>, dim3(grid), dim3(256), 0, st, g);
    const int64_t mn = (int64_t)M * N;
    const unsigned cs_blocks = cout ? (unsigned)((M + 31) / 32) : 0u;  // bias gradient finished in the same launch
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((mn / 4 + 255) / 256) + cs_blocks), dim3(256), 0, st, slab,
                       split, mn, c, out_f32, static_cast<const float*>(colsum), M, cout, out_f32, g.cs_workers);
    return hipGetLastError();
  }
  if (cout) DTA_HIP_CHECK(dta_colsum_partials(colsum, g.cs_workers, M, cout, out_f32, st));
  return hipGetLastError();
}
