// General bf16 GEMM for gfx950 with fused epilogues: the transformer
// projections' forward (y = x W^T + b [, GELU] [, + residual]), input
// gradient (dx = dy W) and weight gradient (dW = dy^T x) -- SURVEY.md N07, the
// GEMMs of nn.Linear at src/distributed_trainer.py:162,164 scaled up to the
// GPT-2 / Llama configs.
//
//   C[M, N] = alpha * sum_k A(m, k) B(n, k)   (+ bias[n], act, + R[m, n])
//
// Operand storage, both bf16 row-major:
//   A: K-major [M][K] (lda)  or  M-major [K][M] (A_T)
//   B: K-major [N][K] (ldb)  or  N-major [K][N] (B_T)
// forward  y = x W^T : A = x [T][K],  B = W [N][K]          (A_T = 0, B_T = 0)
// dgrad   dx = dy W  : A = dy [T][N], B = W [N][K] as [k][n] (A_T = 0, B_T = 1)
// wgrad   dW = dy^T x: A = dy [T][N] as [k][m], B = x as [k][n] (A_T = 1, B_T = 1)
//
// Structure (cdna_hip_programming.md §5): a BM x BN tile per workgroup of 8
// waves (2 x 4), each wave (BM/2) x (BN/4) on v_mfma_f32_16x16x32_bf16; the
// k loop streams 32-deep stages by global_load_lds_dwordx4 (LDS-DMA, no
// staging VGPRs) into a 4-deep LDS ring; the fragments of stage k+1 are read
// from LDS while the MFMAs of stage k run (two register sets), and up to three
// stages of DMA are in flight; the wait before each barrier is a counted vmcnt
// (never 0 inside the loop) and the barrier is a raw s_barrier, so the DMA of
// later stages spans it.
//
// LDS images (all lane-linear for the DMA; the XOR swizzle is applied to the
// per-lane SOURCE address and undone on the read, rule 21):
//  * K-major operand: [rows][32] bf16 = 64-B rows, 16-B chunk c of row r at
//    physical chunk c ^ 3*((r >> 3) & 1).  A fragment read (ds_read_b128, lane
//    l: row l & 15, chunk l >> 4) then hits 16 distinct 16-B bank slots in each
//    of the instruction's four 16-lane bank groups: conflict-free.
//  * M/N-major operand: [32 k][W] bf16 (rows of 2W bytes), chunk c of row k at
//    c ^ 2*((k & 3) | ((k >> 3) & 1) << 2).  Fragments come from
//    ds_read_b64_tr_b16 (two per fragment: k rows 8g..8g+3 and 8g+4..8g+7 of
//    16-lane group g); the 8 rows a 32-lane bank group touches land on 8
//    distinct 32-B bank ranges: conflict-free.
//
// The MFMA is issued as mfma(B-fragment, A-fragment) so each lane's four
// accumulators are FOUR CONSECUTIVE OUTPUT COLUMNS of one row: the epilogue
// adds the bias / applies GELU in fp32 and stores 8-byte bf16x4 pieces.
//
// Tile order: XCD-aware bijective remap of the workgroup id, then groups of 8
// tile rows walked column by column, so the workgroups resident on one XCD
// share A and B panels in its L2.
#include "common.h"

namespace dta {

constexpr int kGbBK = 32;      // k per stage
constexpr int kGbStages = 4;   // LDS ring depth (3 stages in flight)
constexpr int kGbGroupM = 8;   // tile rows per group (L2 panel reuse)

struct GemmBfArgs {
  const bf16* a;
  const bf16* b;
  bf16* c;
  float* c32;           // fp32 output instead of bf16 (nullptr: bf16 to c)
  const bf16* bias;     // [N] or nullptr
  const bf16* res;      // residual [M][ldr] added after rounding, or nullptr
  int64_t lda, ldb, ldc, ldr;
  int M, N, K;
  int tiles_m, tiles_n;
  float alpha;
  int act;              // ACT_NONE / ACT_GELU_TANH / kEpiDGelu
  // CS kernels (weight gradients): the bias gradient db[m] = sum_k A(m, k) (column
  // sums of dy) from an MFMA against an all-ones B fragment in the workgroups of
  // tile column 0 -- bf16 db or fp32 db32 (nullptr both: none)
  bf16* db;
  float* db32;
};

// epilogue of an input gradient through a GELU: C = acc * gelu_tanh'(res) (res = the GELU's input)
constexpr int kEpiDGelu = 16;

__device__ __forceinline__ int kswz(int r) { return ((r >> 3) & 1) * 3; }
__device__ __forceinline__ int mswz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

__device__ __forceinline__ bf16x4 tr4(const char* lds, int byte_off) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(lds + byte_off));
  return __builtin_bit_cast(bf16x4, v);
}

// 16 rows (r0 .. r0+15) x 32 k of a K-major image: lane l -> row r0 + (l & 15), k 8(l >> 4) .. +7
__device__ __forceinline__ bf16x8 frag_k(const char* img, int r0, int lane) {
  const int r = r0 + (lane & 15), c = lane >> 4;
  return *reinterpret_cast<const bf16x8*>(img + r * 64 + 16 * (c ^ kswz(r)));
}

// 16 indices (i0 .. i0+15) x 32 k of an M/N-major image with ROWB-byte rows (same lane map)
template <int ROWB>
__device__ __forceinline__ bf16x8 frag_mn(const char* img, int i0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int k = 8 * g + q;
  const int col = i0 + 4 * p;
  const int off = 16 * ((col >> 3) ^ mswz(k)) + (col & 7) * 2;
  const bf16x4 lo = tr4(img, k * ROWB + off);
  const bf16x4 hi = tr4(img, (k + 4) * ROWB + off);
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int N>
__device__ __forceinline__ void vm_wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// counted wait + barrier: at most `ahead` stages (of L loads each) of this wave still in flight
template <int L>
__device__ __forceinline__ void stage_barrier(int ahead) {
  if (ahead >= 3) vm_wait_n<3 * L>();
  else if (ahead == 2) vm_wait_n<2 * L>();
  else if (ahead == 1) vm_wait_n<L>();
  else vm_wait_n<0>();
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void lds_bar() { asm volatile("s_barrier" ::: "memory"); }

// One BM x BN output tile `t` (row-major tile index of the problem, already
// XCD-remapped) of the problem `g`: the body of gemm_bf16_kernel and of
// gemm_group_kernel.
template <int BM, int BN, bool AT, bool BT, bool PP, bool CS, bool BUF>
__device__ __forceinline__ void gemm_tile(const GemmBfArgs& g, const int t) {
  constexpr int A_BYTES = BM * kGbBK * 2, B_BYTES = BN * kGbBK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int WTM = BM / 2, WTN = BN / 4, MT = WTM / 16, NT = WTN / 16;
  constexpr int AL = BM / 128, BL = BN / 128, L = AL + BL;  // DMA instructions per wave per stage
  __shared__ __attribute__((aligned(1024))) char lds[kGbStages * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  // tile: groups of kGbGroupM tile rows walked column-major
  const int per_group = kGbGroupM * g.tiles_n;
  const int grp = t / per_group, in_g = t - grp * per_group;
  const int gm0 = grp * kGbGroupM, gh = min(kGbGroupM, g.tiles_m - gm0);
  const int tm = gm0 + in_g % gh, tn = in_g / gh;
  const int m0 = tm * BM, n0 = tn * BN;

  // per-lane DMA sources at stage 0 (stage s adds s * step)
  const bf16* srcA[AL];
  const bf16* srcB[BL];
#pragma unroll
  for (int j = 0; j < AL; ++j) {
    const int i = wave * AL + j;
    if constexpr (!AT) {  // K-major: instruction i = rows 16i .. 16i+15, 4 lanes per 64-B row
      const int r = 16 * i + (lane >> 2), c = (lane & 3) ^ kswz(r);
      srcA[j] = g.a + (int64_t)(m0 + r) * g.lda + 8 * c;
    } else {  // M-major: rows of 2*BM bytes, 1024 / (2 BM) rows per instruction
      constexpr int CPR = BM / 8, RPI = 64 / CPR;
      const int r = RPI * i + lane / CPR, c = (lane % CPR) ^ mswz(r);
      srcA[j] = g.a + (int64_t)r * g.lda + m0 + 8 * c;
    }
  }
#pragma unroll
  for (int j = 0; j < BL; ++j) {
    const int i = wave * BL + j;
    if constexpr (!BT) {
      const int r = 16 * i + (lane >> 2), c = (lane & 3) ^ kswz(r);
      srcB[j] = g.b + (int64_t)(n0 + r) * g.ldb + 8 * c;
    } else {
      constexpr int CPR = BN / 8, RPI = 64 / CPR;
      const int r = RPI * i + lane / CPR, c = (lane % CPR) ^ mswz(r);
      srcB[j] = g.b + (int64_t)r * g.ldb + n0 + 8 * c;
    }
  }
  const int64_t stepA = AT ? (int64_t)kGbBK * g.lda : kGbBK;
  const int64_t stepB = BT ? (int64_t)kGbBK * g.ldb : kGbBK;
  // BUF: the pieces through buffer descriptors (32-bit lane offsets, scalar stage step: gemm_k64.hip
  // kFlatDma note); the host takes it when every operand byte lies within 2 GiB of its base
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.a), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.b), 0, 0x7fffffff, 0x00020000);
  unsigned voA[AL], voB[BL];
  if constexpr (BUF) {
#pragma unroll
    for (int j = 0; j < AL; ++j) voA[j] = (unsigned)((srcA[j] - g.a) * 2);
#pragma unroll
    for (int j = 0; j < BL; ++j) voB[j] = (unsigned)((srcB[j] - g.b) * 2);
  }
  auto issue = [&](int s) {
    char* sa = lds + (s & (kGbStages - 1)) * STAGE;
    char* sb = sa + A_BYTES;
    if constexpr (BUF) {
      const unsigned soa = (unsigned)(s * stepA * 2), sob = (unsigned)(s * stepB * 2);
      const unsigned da = lds_addr(lds) + (s & (kGbStages - 1)) * STAGE, db = da + A_BYTES;
#pragma unroll
      for (int j = 0; j < AL; ++j) bglds16(rsA, voA[j], soa, da + (wave * AL + j) * 1024);
#pragma unroll
      for (int j = 0; j < BL; ++j) bglds16(rsB, voB[j], sob, db + (wave * BL + j) * 1024);
    } else {
#pragma unroll
      for (int j = 0; j < AL; ++j) glds16(srcA[j] + s * stepA, sa + (wave * AL + j) * 1024);
#pragma unroll
      for (int j = 0; j < BL; ++j) glds16(srcB[j] + s * stepB, sb + (wave * BL + j) * 1024);
    }
  };

  f32x4 acc[NT][MT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // CS: wave wn sums the A fragments j = wn * JPW .. + JPW - 1 (tile column 0 only)
  constexpr int JPW = MT / 4 > 0 ? MT / 4 : 1;
  f32x4 accb[JPW];
#pragma unroll
  for (int q = 0; q < JPW; ++q) accb[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_cs = CS && tn == 0 && (g.db != nullptr || g.db32 != nullptr);
  const bf16 one = f2bf(1.f);
  const bf16x8 ones = {one, one, one, one, one, one, one, one};
  auto mma_cs = [&](const bf16x8 (&af)[MT]) {
    if constexpr (CS) {
      if (do_cs) {
#pragma unroll
        for (int w = 0; w < 4; ++w)
          if (w == wn && w * JPW < MT) {
#pragma unroll
            for (int q = 0; q < JPW; ++q)
              accb[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[w * JPW + q], accb[q], 0, 0, 0);
          }
      }
    }
  };

  auto frag_a = [&](const char* sa, int j) {
    if constexpr (!AT) return frag_k(sa, wm * WTM + 16 * j, lane);
    else return frag_mn<2 * BM>(sa, wm * WTM + 16 * j, lane);
  };
  auto frag_b = [&](const char* sb, int i) {
    if constexpr (!BT) return frag_k(sb, wn * WTN + 16 * i, lane);
    else return frag_mn<2 * BN>(sb, wn * WTN + 16 * i, lane);
  };
  const int nk = g.K / kGbBK;

  if constexpr (PP) {
    // Ping-pong (cdna_hip_programming.md §5.5 T3-T5): each stage is two phases
    // (half of the wave's B fragments each), and every phase is a load section
    // (ds_reads, LDS-DMA issue, counted vmcnt) and an MFMA section, separated by
    // workgroup barriers.  Waves 4-7 (wm = 1) run ONE BARRIER BEHIND waves 0-3,
    // and each SIMD holds one wave of each group, so while one group multiplies
    // the other loads: the MFMA pipe alternates between the two waves of a SIMD.
    //
    // An MFMA section never waits for LDS reads issued in the load section right
    // before it (that would idle the pipe for a read latency each phase): the A
    // fragments and the first B half of stage k are read in L(k-1, 1) into one of
    // two A register sets, the second B half in L(k, 0).
    //
    // Barrier numbering (group 0; group 1 is +1): L(k,0) #4k+1 M(k,0) #4k+2
    // L(k,1) #4k+3 M(k,1) #4k+4.
    //  * stage k+1 is waited for (vmcnt) in L(k,0) by every wave -> visible after
    //    #4k+2 (group 1's L(k,0)), before its first reads in L(k,1);
    //  * stage k+3 is DMA'd in L(k,1) into the slot of stage k-1, whose last reads
    //    (group 1, L(k-1,0)) retired before group 1's M(k-1,1) ended at #4k+1.
    constexpr int HN = NT / 2;
    bf16x8 afA[MT], afB[MT], b0[HN], b1[HN];
    auto slot = [&](int s) { return lds + (s & (kGbStages - 1)) * STAGE; };
    auto read_a_b0 = [&](int s, bf16x8 (&af)[MT]) {
      const char* sa = slot(s);
#pragma unroll
      for (int j = 0; j < MT; ++j) af[j] = frag_a(sa, j);
#pragma unroll
      for (int i = 0; i < HN; ++i) b0[i] = frag_b(sa + A_BYTES, i);
    };
    auto read_b1 = [&](int s) {
#pragma unroll
      for (int i = 0; i < HN; ++i) b1[i] = frag_b(slot(s) + A_BYTES, HN + i);
    };
    auto mma_half = [&](const bf16x8 (&af)[MT], const bf16x8 (&bh)[HN], int i0) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < HN; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j)
          acc[i0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[i], af[j], acc[i0 + i][j], 0, 0, 0);
      if (i0 == 0) mma_cs(af);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    };
    auto vm_stages = [&](int ahead) {
      if (ahead >= 2) vm_wait_n<2 * L>();
      else if (ahead == 1) vm_wait_n<L>();
      else vm_wait_n<0>();
    };
    const int pre = min(nk, kGbStages - 1);
    for (int s = 0; s < pre; ++s) issue(s);
    vm_stages(pre - 1);  // stage 0 landed (this wave's part)
    lds_bar();
    read_a_b0(0, afA);
    if (wm == 1) lds_bar();
    // one stage; A fragments of stage kt in `ca`, those of kt+1 go to `na`
    auto stage = [&](int kt, const bf16x8 (&ca)[MT], bf16x8 (&na)[MT]) {
      // L(kt, 0)
      if (kt + 1 < nk) vm_stages(min(nk - 1, kt + kGbStages - 2) - (kt + 1));
      read_b1(kt);
      lds_bar();
      // M(kt, 0)
      mma_half(ca, b0, 0);
      lds_bar();
      // L(kt, 1)
      if (kt + kGbStages - 1 < nk) issue(kt + kGbStages - 1);
      read_a_b0(kt + 1, na);  // (past the last stage: a stale slot, never multiplied; unconditional keeps
                              //  the LDS-read count static so hipcc's lgkmcnt waits stay partial)
      lds_bar();
      // M(kt, 1)
      mma_half(ca, b1, HN);
      lds_bar();
    };
    for (int kt = 0; kt < nk; kt += 2) {
      stage(kt, afA, afB);
      if (kt + 1 < nk) stage(kt + 1, afB, afA);
    }
    if (wm == 0) lds_bar();  // same barrier count for both groups
  } else {
    // fragments of one stage (two named sets: stage kt+1 is read while stage kt multiplies)
    auto read = [&](int s, bf16x8 (&af)[MT], bf16x8 (&bfr)[NT]) {
      const char* sa = lds + (s & (kGbStages - 1)) * STAGE;
      const char* sb = sa + A_BYTES;
#pragma unroll
      for (int j = 0; j < MT; ++j) af[j] = frag_a(sa, j);
#pragma unroll
      for (int i = 0; i < NT; ++i) bfr[i] = frag_b(sb, i);
    };
    auto mma = [&](const bf16x8 (&af)[MT], const bf16x8 (&bfr)[NT]) {
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[i], af[j], acc[i][j], 0, 0, 0);
      mma_cs(af);
    };
    // Ring: stage s in slot s % 4.  Iteration kt: [wait stage kt+1, barrier] [DMA stage
    // kt+4 into slot kt % 4 -- stage kt's fragments were read in iteration kt-1 and the
    // barrier's lgkmcnt(0) retired those reads on every wave] [read stage kt+1] [MFMA kt].
    const int pre = min(nk, kGbStages);
    for (int s = 0; s < pre; ++s) issue(s);
    stage_barrier<L>(pre - 1);  // stage 0 landed everywhere
    bf16x8 afA[MT], bfA[NT], afB[MT], bfB[NT];
    read(0, afA, bfA);
    auto body = [&](int kt, const bf16x8 (&ca)[MT], const bf16x8 (&cb)[NT], bf16x8 (&na)[MT], bf16x8 (&nb)[NT]) {
      if (kt + 1 < nk) {
        stage_barrier<L>(min(nk - 1, kt + kGbStages - 1) - (kt + 1));
        if (kt + kGbStages < nk) issue(kt + kGbStages);
        read(kt + 1, na, nb);
      }
      mma(ca, cb);
    };
    for (int kt = 0; kt < nk; kt += 2) {
      body(kt, afA, bfA, afB, bfB);
      if (kt + 1 < nk) body(kt + 1, afB, bfB, afA, bfA);
    }
  }

  // epilogue: lane holds rows m = .. + (lane & 15), columns n = .. + 4 (lane >> 4) + r (r = 0..3)
  const int mrow = m0 + wm * WTM + (lane & 15);
  const int ncol = n0 + wn * WTN + 4 * (lane >> 4);
  if constexpr (CS) {
    if (do_cs && wn * JPW < MT && (lane >> 4) == 0) {  // the four columns of accb are equal
#pragma unroll
      for (int q = 0; q < JPW; ++q) {
        const int m = mrow + 16 * (wn * JPW + q);
        if (g.db32) g.db32[m] = accb[q][0];
        else g.db[m] = f2bf(accb[q][0]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int n = ncol + 16 * i;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (g.bias) {
      const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(g.bias + n);
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = bf2f(b4[r]);
    }
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int m = mrow + 16 * j;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = fmaf(acc[i][j][r], g.alpha, bv[r]);
        if (g.act == ACT_GELU_TANH) v[r] = act_fwd(ACT_GELU_TANH, v[r]);
      }
      if (g.c32) {
        *reinterpret_cast<float4*>(g.c32 + (int64_t)m * g.ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
        continue;
      }
      if (g.act == kEpiDGelu) {  // dgrad through the GELU: one rounding (of the product)
        const bf16x4 h4 = *reinterpret_cast<const bf16x4*>(g.res + (int64_t)m * g.ldr + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= act_bwd(ACT_GELU_TANH, bf2f(h4[r]));
      } else if (g.res) {  // residual stream: y = round(round(linear) + res), as two bf16 ops would give
        const bf16x4 r4 = *reinterpret_cast<const bf16x4*>(g.res + (int64_t)m * g.ldr + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = bf2f(f2bf(v[r])) + bf2f(r4[r]);
      }
      *reinterpret_cast<bf16x4*>(g.c + (int64_t)m * g.ldc + n) = bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
    }
  }
}

template <int BM, int BN, bool AT, bool BT, bool PP, bool BUF>
__global__ void __launch_bounds__(512) gemm_bf16_kernel(GemmBfArgs g) {
  gemm_tile<BM, BN, AT, BT, PP, false, BUF>(g, xcd_remap(blockIdx.x, g.tiles_m * g.tiles_n));
}

// every byte an operand spans within 2 GiB of its base: the buffer-descriptor DMA form applies
static inline bool bf_fits_2g(int64_t rows_minus1, int64_t ld, int64_t cols) {
  return 2 * (rows_minus1 * ld + cols) < 0x7fffffffLL;
}

// Grouped weight gradients: several independent problems (dW_i = dy_i^T x_i, each with
// its bias gradient) in ONE launch of 256 x 256 tiles over the full token reduction --
// no split-K, no fp32 slabs.  The tiles of all problems form one list (problem-major,
// XCD-remapped so each XCD takes a contiguous run: neighbouring tiles of one problem,
// whose dy / x panels its L2 then shares).  Used for the GPT-2-sized weight gradients,
// deferred and batched across Linear layers (ops/lm.py).
constexpr int kGroupMax = 16;
struct GemmGroupArgs {
  int n;
  int tile_start[kGroupMax + 1];
  GemmBfArgs p[kGroupMax];
};

template <bool BUF>
__global__ void __launch_bounds__(512) gemm_group_kernel(GemmGroupArgs ga) {
  const int t = xcd_remap(blockIdx.x, ga.tile_start[ga.n]);
  int q = 0;
  while (q + 1 < ga.n && t >= ga.tile_start[q + 1]) ++q;
  gemm_tile<256, 256, true, true, true, true, BUF>(ga.p[q], t - ga.tile_start[q]);
}

template <int BM, int BN, bool AT, bool BT>
static hipError_t launch_bf(const GemmBfArgs& g, hipStream_t st) {
  // static LDS: 4 x (BM + BN) x 64 B (128 KiB at 256 x 256: one workgroup per CU)
  constexpr bool PP = BM == 256 && BN == 256;  // ping-pong schedule for the big tile
  const bool buf = (AT ? bf_fits_2g(g.K - 1, g.lda, g.M) : bf_fits_2g(g.M - 1, g.lda, g.K)) &&
                   (BT ? bf_fits_2g(g.K - 1, g.ldb, g.N) : bf_fits_2g(g.N - 1, g.ldb, g.K));
  if (buf)
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, AT, BT, PP, true>), dim3(g.tiles_m * g.tiles_n), dim3(512), 0, st, g);
  else
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, AT, BT, PP, false>), dim3(g.tiles_m * g.tiles_n), dim3(512), 0, st, g);
  return hipGetLastError();
}

template <int BM, int BN>
static hipError_t launch_tile(const GemmBfArgs& g, bool at, bool bt, hipStream_t st) {
  if (!at && !bt) return launch_bf<BM, BN, false, false>(g, st);
  if (!at && bt) return launch_bf<BM, BN, false, true>(g, st);
  if (at && bt) return launch_bf<BM, BN, true, true>(g, st);
  return launch_bf<BM, BN, true, false>(g, st);
}

}  // namespace dta

using namespace dta;

// Tile choice: minimise (rounds of resident workgroups) x (tile work / tile efficiency).
// tile = 0: auto; 1: 256x256, 2: 256x128, 3: 128x128 (when it divides the problem).
int dta_gemm_bf16_tile(int M, int N, int K, int tile) {
  static const int bm[4] = {0, 256, 256, 128}, bn[4] = {0, 256, 128, 128};
  static const double eff[4] = {0, 1.0, 0.86, 0.72};   // relative MFMA efficiency of the tile shapes
  static const int per_cu[4] = {0, 1, 1, 2};          // resident workgroups per CU (LDS ring size)
  if (K % kGbBK || K < kGbBK) return 0;
  if (tile) return (M % bm[tile] == 0 && N % bn[tile] == 0) ? tile : 0;
  int best = 0;
  double best_t = 1e30;
  for (int t = 1; t <= 3; ++t) {
    if (M % bm[t] || N % bn[t]) continue;
    const int tiles = (M / bm[t]) * (N / bn[t]);
    const int slots = 256 * per_cu[t];
    const int rounds = (tiles + slots - 1) / slots;
    // a round costs one tile's time on a CU shared by per_cu workgroups
    const double tt = rounds * (double)bm[t] * bn[t] * per_cu[t] / eff[t];
    if (tt < best_t * 0.999) {
      best_t = tt;
      best = t;
    }
  }
  return best;
}

hipError_t dta_gemm_bf16(const void* a, int64_t lda, bool a_t, const void* b, int64_t ldb, bool b_t, void* c,
                         float* c32, int64_t ldc, int M, int N, int K, float alpha, const void* bias, int act,
                         const void* res, int64_t ldr, int tile, hipStream_t st) {
  tile = dta_gemm_bf16_tile(M, N, K, tile);
  if (!tile || N % 8 || (!c && !c32)) return hipErrorInvalidValue;
  GemmBfArgs g{};
  g.a = static_cast<const bf16*>(a);
  g.b = static_cast<const bf16*>(b);
  g.c = static_cast<bf16*>(c);
  g.c32 = c32;
  g.bias = static_cast<const bf16*>(bias);
  g.res = static_cast<const bf16*>(res);
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.ldr = ldr;
  g.M = M;
  g.N = N;
  g.K = K;
  g.alpha = alpha;
  g.act = act;
  switch (tile) {
    case 1:
      g.tiles_m = M / 256;
      g.tiles_n = N / 256;
      return launch_tile<256, 256>(g, a_t, b_t, st);
    case 2:
      g.tiles_m = M / 256;
      g.tiles_n = N / 128;
      return launch_tile<256, 128>(g, a_t, b_t, st);
    default:
      g.tiles_m = M / 128;
      g.tiles_n = N / 128;
      return launch_tile<128, 128>(g, a_t, b_t, st);
  }
}

// n problems dW_i[M_i][N_i] (bf16, row stride ldc_i) = A_i^T B_i with A_i = dy [K_i][M_i]
// (lda_i), B_i = x [K_i][N_i] (ldb_i); db_i (bf16 [M_i], or nullptr) = column sums of A_i.
// Every M_i, N_i a multiple of 256, K_i of 32.
int dta_gemm_group_max() { return kGroupMax; }

hipError_t dta_gemm_wgrad_group(int n, const void* const* a, const int64_t* lda, const void* const* b,
                                const int64_t* ldb, void* const* c, const int64_t* ldc, const int* M, const int* N,
                                const int* K, void* const* db, hipStream_t st) {
  if (n < 1 || n > kGroupMax) return hipErrorInvalidValue;
  GemmGroupArgs ga{};
  ga.n = n;
  int total = 0;
  for (int i = 0; i < n; ++i) {
    if (M[i] % 256 || N[i] % 256 || K[i] % kGbBK || K[i] < kGbBK) return hipErrorInvalidValue;
    GemmBfArgs& g = ga.p[i];
    g.a = static_cast<const bf16*>(a[i]);
    g.b = static_cast<const bf16*>(b[i]);
    g.c = static_cast<bf16*>(c[i]);
    g.lda = lda[i];
    g.ldb = ldb[i];
    g.ldc = ldc[i];
    g.M = M[i];
    g.N = N[i];
    g.K = K[i];
    g.tiles_m = M[i] / 256;
    g.tiles_n = N[i] / 256;
    g.alpha = 1.f;
    g.act = ACT_NONE;
    g.db = static_cast<bf16*>(db[i]);
    ga.tile_start[i] = total;
    total += g.tiles_m * g.tiles_n;
  }
  ga.tile_start[n] = total;
  bool buf = true;
  for (int i = 0; i < n; ++i)
    buf = buf && bf_fits_2g(K[i] - 1, lda[i], M[i]) && bf_fits_2g(K[i] - 1, ldb[i], N[i]);
  if (buf)
    hipLaunchKernelGGL(gemm_group_kernel<true>, dim3(total), dim3(512), 0, st, ga);
  else
    hipLaunchKernelGGL(gemm_group_kernel<false>, dim3(total), dim3(512), 0, st, ga);
  return hipGetLastError();
}
