// bf16 GEMM for gfx950 with 64-deep k stages, a phase-interleaved half-tile
// DMA pipeline and fused epilogues -- the transformer projections' forward
// (y = x W^T + b [, GELU with a dual store of pre-activation and activation]
// [, + residual]), input gradient (dx = dy W [, * gelu'(h)]) and weight
// gradient (dW = dy^T x): SURVEY.md N07, the GEMMs of nn.Linear at
// src/distributed_trainer.py:162,164 scaled to the GPT-2 / Llama configs.
//
//   C[M, N] = alpha * sum_k A(m, k) B(n, k)   (+ bias[n], epilogue)
//
// Operand storage (bf16, unit inner stride):
//   A: K-major [M][K] (lda)  or  M-major [K][M] (AT)
//   B: K-major [N][K] (ldb)  or  N-major [K][N] (BT)
//
// Structure (cdna_hip_programming.md §5 "The 256² 8-phase template", T1-T5):
//  * BM x BN tile per workgroup of 2 x WC waves; waves are laid out so that
//    the A operand's two HALF-TILES (rows [0, BM/2) and [BM/2, BM)) and B's two
//    half-tiles each feed ONE quadrant phase of every wave: wave (wr, wc) owns
//    rows {mh * BM/2 + wr * BM/4 + [0, BM/4)} and columns
//    {nh * BN/2 + wc * BN/(2 WC) + [0, BN/(2 WC))} for mh, nh in {0, 1}.
//  * Two K-loop forms (template PH): the two-phase form, the default for the 8-wave
//    tiles (ids 5, 6, 8), reads A-top + both B halves, then A-bottom, and runs 32
//    MFMAs per cluster between two barriers -- half the barriers of the four-phase
//    form, 3-11 % faster at every GPT-2 / Llama shape with the stagger below; both
//    forms keep every wait three or more half-tiles deep.  The four-phase form:
//  * A K-tile (64 deep) is four phases; phase = [ds_read of the quadrant's
//    fragments | LDS-DMA (global_load_lds_dwordx4) of ONE half-tile of a later
//    K-tile | counted vmcnt] -> s_barrier -> lgkmcnt(0) -> 16 MFMAs -> s_barrier:
//      P1 read A-top, B-left   DMA right (t+1)     MFMA top x left
//      P2 read B-right         DMA bottom (t+1)    vmcnt(2LA+2LB)  MFMA top x right
//      P3 read A-bottom        DMA top (t+2)       MFMA bottom x right
//      P4 (registers)          DMA left (t+2)      vmcnt(2LA+LB)   MFMA bottom x left
//    Two LDS buffers (K-tile t in buffer t & 1).  Every half-tile is restaged
//    two or more phases after its last read (safe with the wave-group stagger
//    below: a phase's reads are retired by its lgkmcnt(0) before its second
//    barrier); every wait retires the half-tiles read one phase later or
//    more, and leaves three half-tiles in flight -- vmcnt is never 0 in the
//    loop, barriers are raw s_barrier (the LDS-DMA spans them).
//  * Waves 4-7 run one barrier behind waves 0-3 (stagger, MI355X_MICROARCH.md
//    "Two waves per SIMD" item 9): while one wave of a SIMD multiplies, its
//    partner loads.  MFMA clusters are pinned between the barriers with
//    s_setprio / sched_barrier (T5).
//  * LDS images are lane-linear for the DMA; the XOR swizzle goes on the
//    per-lane SOURCE address and is undone on the read (rule 21):
//      K-major (128-B rows of 64 k):  chunk c of row r at c ^ (r & 7)
//        -> ds_read_b128 fragment reads conflict-free;
//      M/N-major (64 k-rows of 2 x BM/2 bytes): chunk ch of k-row k at
//        ch ^ ((k&3)<<2 | (k>>2)&3) (256-B rows) or ch ^ ((k>>1&1)<<1 | (k>>3&1)<<2)
//        (128-B rows) -> ds_read_b64_tr_b16 reads conflict-free (verified with
//        scripts/lds_banks.py's bank model).
//  * v_mfma_f32_16x16x32_bf16 (on random data it holds a higher clock than
//    32x32x16 at equal cycles per FLOP: MI355X_MICROARCH.md "DVFS give-back"
//    item 7), issued as mfma(B, A) so each lane's four accumulators are four
//    consecutive output COLUMNS: the epilogue stores bf16x4 pieces.
//  * Out-of-range K-tiles of the pipeline's tail are DMA'd from the last
//    K-tile (never read): the vmcnt counts stay static; drained before exit.
//    (A persistent variant -- each workgroup walking several tiles with the
//    DMA running across tile boundaries -- measured slower at every GPT-2 and
//    Llama shape: 51 vs 46 us on the GPT-2 qkv forward, 136 vs 92 us on its
//    weight gradient; the epilogue inside the K loop costs registers and
//    scheduling freedom.)
//  * Tile order: XCD-aware bijective remap, then groups of 8 tile rows walked
//    column by column (L2 panel reuse on each XCD).
//  * Measured and dropped (round 3): a 4-wave 256x256 tile, one wave per SIMD with a 128x128 output each
//    (256 AGPR accumulators, two thirds of the LDS read bytes per FLOP), 32-deep stages in a 4- or
//    5-buffer LDS ring, the next stage's fragment reads and the DMA interleaved between the 64 MFMAs of
//    a stage: 989-1145 TF/s vs 1303-1413 for the 8-wave two-phase tile at Llama shapes.  In-kernel stamps
//    put 88 % of its stage in the MFMA stream at ~22 cycles per 16-cycle MFMA: the LDS-DMA pieces'
//    issue cost (8 per stage, ~60 cycles each: MI355X_MICROARCH.md) lands on the only wave of the
//    SIMD, where the 8-wave form hands it to the partner wave.
#pragma once
// (the device side of csrc/gemm_k64.hip, shared with csrc/gemm_k64_sk.hip: the stream-K instantiations build
// in their own translation unit, in parallel)
#include "common.h"
#include "gemm_epi.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace dta {
namespace k64 {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// DTA_K64_DMA_IN_MFMA (diagnostic builds, scripts/k64_dim_probe.hip): the two-phase loop issues each phase's
// LDS-DMA pieces inside the phase's MFMA cluster (spread between the MFMAs) instead of in its read phase.
#ifndef DTA_K64_DMA_IN_MFMA
#define DTA_K64_DMA_IN_MFMA 0
#endif

template <int N, int I = 0, typename F>
__device__ __forceinline__ void k64_static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    k64_static_for<N, I + 1>(f);
  }
}

#ifdef DTA_K64_STAMP
// s_memtime with its lgkmcnt(0) in ONE statement (cdna_hip_programming.md "In-kernel stamps"); the
// diagnostic build's run time is never quoted, only the segment shares
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define K64_STAMP(i)                \
  do {                              \
    const unsigned long long n_ = stamp_now(); \
    seg[i] += n_ - t_prev;          \
    t_prev = n_;                    \
  } while (0)
#else
#define K64_STAMP(i) \
  do {               \
  } while (0)
#endif

#ifdef DTA_K64_TIMELINE
// diagnostic build (scripts/k64_timeline.hip): per wave, the device real-time clock (100 MHz, one clock for
// every CU) at kernel entry (0), after the K loop's prologue (1), after the K loop (2) and after the epilogue's
// stores have drained (3), plus the wave's HW_ID (4), XCC_ID (5) and the time its epilogue stores were all
// issued (6) -- where a tile's time goes outside the loop (8 slots per wave)
__device__ __forceinline__ unsigned long long k64_rt() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define K64_TL(i, v)                                                                         \
  do {                                                                                     \
    if ((threadIdx.x & 63) == 0) g.stamps[((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (i)] = (v); \
  } while (0)
#else
#define K64_TL(i, v) \
  do {               \
  } while (0)
#endif

__device__ __forceinline__ bf16x4 tr4(const char* lds, int byte_off) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(lds + byte_off));
  return __builtin_bit_cast(bf16x4, v);
}

// chunk swizzle of an M/N-major image with RB-byte k-rows
template <int RB>
__device__ __forceinline__ int mswz(int k) {
  if constexpr (RB == 256) return ((k & 3) << 2) | ((k >> 2) & 3);
  else return (((k >> 1) & 1) << 1) | (((k >> 3) & 1) << 2);
}

// fragment (16 rows r0.., k 32 kk .. +31) of a K-major half image: lane l -> row r0 + (l & 15), k 8 (l >> 4) ..
__device__ __forceinline__ bf16x8 frag_k(const char* img, int r0, int kk, int lane) {
  const int r = r0 + (lane & 15), c = 4 * kk + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(img + r * 128 + 16 * (c ^ (r & 7)));
}

// the same fragment (16 indices i0.., k 32 kk ..) of an M/N-major half image with RB-byte k-rows
template <int RB>
__device__ __forceinline__ bf16x8 frag_mn(const char* img, int i0, int kk, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int k = 32 * kk + 8 * g + q;
  const int col = i0 + 4 * p, ch = col >> 3, w = (col & 7) * 2;
  const bf16x4 lo = tr4(img, k * RB + 16 * (ch ^ mswz<RB>(k)) + w);
  const bf16x4 hi = tr4(img, (k + 4) * RB + 16 * (ch ^ mswz<RB>(k + 4)) + w);
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// WR x WC waves (WR = 2 but for the 192-wide tiles' 4 x 2 grid: a 96-column half over 2 wave columns)
template <int BM, int BN, int WC, bool AT, bool BT, int WR = 2>
struct Cfg {
  static constexpr int NW = WR * WC, NTHR = 64 * NW;
  static constexpr int HA = BM / 2, HB = BN / 2;                  // half-tile rows / columns
  static constexpr int A_HALF = HA * BK * 2, B_HALF = HB * BK * 2;  // bytes
  static constexpr int LA = A_HALF / (NTHR * 16), LB = B_HALF / (NTHR * 16);  // DMA per thread per half
  // BJ: a B half is not a whole number of 1 KiB pieces per wave (BN 192 over 8 waves: 12 pieces): both
  // halves go as ONE 24-piece image (they are always staged together in the two-phase loop)
  static constexpr bool BJ = B_HALF % (NTHR * 16) != 0;
  static constexpr int LB2 = 2 * B_HALF / (NTHR * 16);             // B pieces per thread per K-tile
  static constexpr int BUF = 2 * A_HALF + 2 * B_HALF;
  static constexpr int MTH = HA / (16 * WR), NTH = HB / (16 * WC);  // fragments per wave per half
  static constexpr int RBA = 2 * HA, RBB = 2 * HB;                 // M/N-major image row bytes
  static constexpr int CPR = BN / 8;                               // 16-B chunks per row of a bf16 C tile image
  static_assert(LA >= 1 && LB2 >= 2 && MTH >= 1 && NTH >= 1, "tile too small for the workgroup");
  static_assert(A_HALF % (NTHR * 16) == 0 && (2 * B_HALF) % (NTHR * 16) == 0, "whole DMA pieces per wave");
  static_assert(HA % (16 * WR) == 0 && HB % (16 * WC) == 0, "whole fragments per wave");
  static_assert(!AT || RBA == 256 || RBA == 128, "M-major A: BM 256 or 128");
  static_assert(!BT || RBB == 256 || RBB == 128, "N-major B: BN 256 or 128");
  static_assert(!BJ || !BT, "joint B staging: K-major B only");
};

// chunk swizzle of a C tile image row (CPR chunks): the row index mod CPR for the power-of-two widths, its
// low three bits for CPR = 24 (an XOR below 8 keeps a chunk inside its group of 8: a permutation of [0, 24))
template <int CPR>
__device__ __forceinline__ int cswz(int row) {
  if constexpr ((CPR & (CPR - 1)) == 0) return row % CPR;
  else return row & 7;
}

// Stream-K (SK): the grid's G workgroups split the problem's tiles x K-tiles "units" into equal runs of
// `span` >= ceil(nk / 2) units, so every CU gets the same work whatever the tile count (GPT-2's N = 768
// input gradients are 192 tiles of 256 x 128 for 256 CUs; Llama's qkv weight gradient 384 of 256 x 256).
// A tile whose K range is cut between workgroups (at most three, by the span bound) is finished by the
// LAST of them to arrive: each contributor stores its fp32 accumulators write-through (sc1, 16 B) into its
// own slab, drains them (vmcnt(0) in every wave), and one lane adds to the tile's counter (agent scope);
// the workgroup whose add returns n - 1 reads the other slabs with sc1 loads, sums the parts in K order
// (((p0 + p1) + p2): the same bits whoever arrives last -- fp32 addition commutes) and runs the normal
// epilogue, then re-zeroes the counter (zeroed once at allocation; cdna_hip_programming.md split-K
// in-launch reduction, the sc1 form).  No workgroup ever waits for another.
struct SkArgs {
  float* ws;         // [G][2][BM * BN] fp32 slabs: a workgroup's first (slot 0) and last (slot 1) segment
  int* cnt;          // [tiles] arrival counters, zero between launches
  int span;          // units (K-tiles) per workgroup
};

// STG (one bf16 output): the epilogue goes through the LDS as a whole BM x BN bf16 tile image (in the LDS
// the K loop used: the image is at most its size) and leaves as whole 2 BN-byte rows -- instead of one 8-B
// store per lane per fragment (16 rows x 32 B per instruction).  Measured (scripts/bench_w4.py, 256 x 256):
// Llama o-proj forward 204.6 -> 188.6 us, LM head forward 6110 -> 5806 us (hipBLASLt 5830), GPT-2 qkv forward
// 59.2 -> 44.8 us.
// DSW: the EPI_DSWIGLU instantiation (a compile-time form: its two-round epilogue in the shared body cost
// every other kernel registers -- 256 VGPRs and scratch spills at the 256 x 256 tile)
template <int BM, int BN, int WC, bool AT, bool BT, int PH, bool BUF, bool CS, bool STG = false, bool DSW = false,
          int WR = 2, bool SK = false>
__device__ __forceinline__ void k64_body(const Args& g, const int t, const int kb = 0, const int ke = 0,
                                         const SkArgs* sk = nullptr, const int wsk = 0, const int slot = 0) {
  static_assert(!SK || (PH == 2 && !CS && !DSW), "stream-K: two-phase loop, plain / fused epilogues");
  static_assert(!DSW || STG, "the SwiGLU-backward epilogue is LDS-staged only");
  static_assert(!CS || (PH == 2 && AT), "bias-gradient column sums: two-phase loop, M-major A (weight gradients)");
  static_assert(!STG || BM * BN * 2 <= 2 * Cfg<BM, BN, WC, AT, BT, WR>::BUF, "staged epilogue: the tile image fits the LDS");
  using C = Cfg<BM, BN, WC, AT, BT, WR>;
  constexpr int HA = C::HA, HB = C::HB, LA = C::LA, LB = C::LB, LB2 = C::LB2, MTH = C::MTH, NTH = C::NTH, NW = C::NW;
  constexpr bool BJ = C::BJ;
  static_assert(!BJ || PH == 2, "joint B staging: two-phase loop only");
  constexpr bool STAG = NW == 8;  // two waves per SIMD: stagger the halves (waves 4-7 one barrier behind)
  static_assert(!STAG || WC == 4 || WR == 4, "stagger groups: waves 0-3 / 4-7");
  __shared__ __attribute__((aligned(1024))) char lds[2 * C::BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WC, wc = wave % WC;
  const bool lag = wave >= NW / 2;  // (STAG) the lagging wave group

  // ---- tile (t: this problem's tile index, XCD-remapped by the caller) ----
  const int per_group = kGroupM * g.tiles_n;
  const int grp = t / per_group, in_g = t - grp * per_group;
  const int gm0 = grp * kGroupM, gh = min(kGroupM, g.tiles_m - gm0);
  const int m0 = (gm0 + in_g % gh) * BM, n0 = (in_g / gh) * BN;
  const int nk_all = g.K / BK;
  // SK: this workgroup's K-tiles [kb, ke) of the tile (the DMA offsets start at kb); else all of them
  const int kofs = SK ? kb : 0, nk = SK ? ke - kb : nk_all;

  // ---- per-lane DMA sources of K-tile 0 (half h: rows / columns [h * H, (h+1) * H)) ----
  // half index: 0 top, 1 bottom, 2 left, 3 right; LDS: buffer b at b * BUF, [top|bottom|left|right]
  // B DMA groups: the two halves, or (BJ) one group of both halves' rows as one image (the halves are
  // contiguous in the LDS and 96 rows is a multiple of the swizzle's 8, so a piece's rows need no split)
  constexpr int NBH = BJ ? 1 : 2, LBG = BJ ? LB2 : LB;
  const bf16* srcA[2][LA];
  const bf16* srcB[NBH][LBG];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int j = 0; j < LA; ++j) {
      const int i = j * NW + wave;  // 1 KiB piece of the half image
      if constexpr (!AT) {
        const int r = 8 * i + (lane >> 3), c = (lane & 7) ^ (r & 7);
        srcA[h][j] = g.a + (int64_t)(m0 + h * HA + r) * g.lda + 8 * c;
      } else {
        constexpr int CPR = C::RBA / 16, RPI = 64 / CPR;
        const int k = RPI * i + lane / CPR, ch = (lane % CPR) ^ mswz<C::RBA>(k);
        srcA[h][j] = g.a + (int64_t)k * g.lda + m0 + h * HA + 8 * ch;
      }
    }
  }
#pragma unroll
  for (int h = 0; h < NBH; ++h) {
#pragma unroll
    for (int j = 0; j < LBG; ++j) {
      const int i = j * NW + wave;
      if constexpr (!BT) {
        const int r = 8 * i + (lane >> 3), c = (lane & 7) ^ (r & 7);
        srcB[h][j] = g.b + (int64_t)(n0 + h * HB + r) * g.ldb + 8 * c;
      } else {
        constexpr int CPR = C::RBB / 16, RPI = 64 / CPR;
        const int k = RPI * i + lane / CPR, ch = (lane % CPR) ^ mswz<C::RBB>(k);
        srcB[h][j] = g.b + (int64_t)k * g.ldb + n0 + h * HB + 8 * ch;
      }
    }
  }
  const int64_t stepA = AT ? (int64_t)BK * g.lda : BK;
  const int64_t stepB = BT ? (int64_t)BK * g.ldb : BK;
  // BUF: the same pieces through buffer descriptors (32-bit lane offsets, scalar K-step); the host
  // takes this form only when every operand byte lies within 4 GiB of its base
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.a), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.b), 0, 0x7fffffff, 0x00020000);
  unsigned voA[2][LA], voB[NBH][LBG];
  if constexpr (BUF) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int j = 0; j < LA; ++j) voA[h][j] = (unsigned)((srcA[h][j] - g.a) * 2);
    }
#pragma unroll
    for (int h = 0; h < NBH; ++h) {
#pragma unroll
      for (int j = 0; j < LBG; ++j) voB[h][j] = (unsigned)((srcB[h][j] - g.b) * 2);
    }
  }
  const unsigned lds0 = lds_addr(lds);
  // LDS layout ILV: [A-top p0 | A-top p1 | A-bottom p0 | A-bottom p1 | B-left p0 | B-left p1 | B-right p0
  // | B-right p1] (p = K-tile parity): with the two-phase loop unrolled by two K-tiles the parity is a
  // compile-time constant and every fragment read is a loop-invariant lane base + an immediate offset
  // (no per-K-tile address arithmetic: 36 VALU per K-tile in the M/N-major layouts before); otherwise
  // [p0: A-top | A-bottom | B-left | B-right][p1: ...] with runtime parity
  // (the 256 x 256 tile with buffer-descriptor DMA only: measured 0-9 % faster there at every GPT-2 /
  // Llama shape and up to 14 % on the long-K weight gradients, while the 128-wide tiles lost ~10 % at
  // K = 768 and the flat-DMA 256 x 256 form spilled; profiles/k64_buffer_dma.jsonl notes)
  constexpr bool ILV = BM == 256 && BN == 256 && BUF;
  auto aoff = [&](int h, int par) { return ILV ? (2 * h + par) * C::A_HALF : par * C::BUF + h * C::A_HALF; };
  auto boff = [&](int h, int par) {
    return ILV ? 4 * C::A_HALF + (2 * h + par) * C::B_HALF : par * C::BUF + 2 * C::A_HALF + h * C::B_HALF;
  };
  auto dma_a = [&](int h, int kt) {  // A half h of K-tile kt (past the end: the last K-tile, never read)
    const int ks = kofs + min(kt, nk - 1);
    char* dst = lds + aoff(h, kt & 1);
    if constexpr (BUF) {
      const unsigned so = (unsigned)(ks * stepA * 2), d0 = lds0 + aoff(h, kt & 1);
#pragma unroll
      for (int j = 0; j < LA; ++j) bglds16(rsA, voA[h][j], so, d0 + (j * NW + wave) * 1024);
    } else {
#pragma unroll
      for (int j = 0; j < LA; ++j) glds16(srcA[h][j] + ks * stepA, dst + (j * NW + wave) * 1024);
    }
  };
  auto dma_b = [&](int h, int kt) {  // (BJ: h = 0 stages both halves, h = 1 nothing)
    if (BJ && h) return;
    const int ks = kofs + min(kt, nk - 1);
    char* dst = lds + boff(h, kt & 1);
    if constexpr (BUF) {
      const unsigned so = (unsigned)(ks * stepB * 2), d0 = lds0 + boff(h, kt & 1);
#pragma unroll
      for (int j = 0; j < LBG; ++j) bglds16(rsB, voB[BJ ? 0 : h][j], so, d0 + (j * NW + wave) * 1024);
    } else {
#pragma unroll
      for (int j = 0; j < LBG; ++j) glds16(srcB[BJ ? 0 : h][j] + ks * stepB, dst + (j * NW + wave) * 1024);
    }
  };

  // ---- fragment reads: the wave's quadrant of a half ----
  auto read_a = [&](bf16x8 (&af)[MTH][2], int kt, int h) {
    const char* img = lds + aoff(h, kt & 1);
#pragma unroll
    for (int jj = 0; jj < MTH; ++jj)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int r0 = wr * (HA / WR) + 16 * jj;
        if constexpr (!AT) af[jj][kk] = frag_k(img, r0, kk, lane);
        else af[jj][kk] = frag_mn<C::RBA>(img, r0, kk, lane);
      }
  };
  auto read_b = [&](bf16x8 (&bf)[NTH][2], int kt, int h) {
    const char* img = lds + boff(h, kt & 1);
#pragma unroll
    for (int ii = 0; ii < NTH; ++ii)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c0 = wc * (HB / WC) + 16 * ii;
        if constexpr (!BT) bf[ii][kk] = frag_k(img, c0, kk, lane);
        else bf[ii][kk] = frag_mn<C::RBB>(img, c0, kk, lane);
      }
  };

  f32x4 acc[2 * NTH][2 * MTH];
#pragma unroll
  for (int i = 0; i < 2 * NTH; ++i)
#pragma unroll
    for (int j = 0; j < 2 * MTH; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const bf16x8 (&af)[MTH][2], const bf16x8 (&bf)[NTH][2], int mh, int nh) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ii = 0; ii < NTH; ++ii)
#pragma unroll
        for (int jj = 0; jj < MTH; ++jj)
          acc[nh * NTH + ii][mh * MTH + jj] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ii][kk], af[jj][kk], acc[nh * NTH + ii][mh * MTH + jj], 0,
                                                      0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
  // CS (tile column 0 of a weight-gradient problem): db[m] = sum_k A(m, k) from MFMAs against an
  // all-ones B fragment -- the four waves sharing A rows split the row fragments (wave wc takes
  // fragment jj = wc of each half: 4 extra MFMAs per K-tile, +6 % on those workgroups only)
  const bool do_cs = CS && g.db != nullptr && n0 == 0;
  f32x4 accb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  auto mma_cs = [&](const bf16x8 (&af)[MTH][2], int mh) {
    if constexpr (CS) {
      if (do_cs) {
        const bf16 one = f2bf(1.f);
        const bf16x8 ones = {one, one, one, one, one, one, one, one};
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jj = 0; jj < MTH; ++jj)
          if (jj == wc) {
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) accb[mh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[jj][kk], accb[mh], 0, 0, 0);
          }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  bf16x8 af[MTH][2], b0[NTH][2], b1[NTH][2];
  if constexpr (PH == 4) {
  // ---- prologue: K-tile 0 whole + top / left of K-tile 1; retire top, left, right of 0 ----
  dma_a(0, 0);
  dma_b(0, 0);
  dma_b(1, 0);
  dma_a(1, 0);
  dma_a(0, 1);
  dma_b(0, 1);
  vm_wait<2 * LA + LB>();
  bar();
  if constexpr (STAG) {
    if (lag) bar();
  }

  for (int kt = 0; kt < nk; ++kt) {
    // P1
    read_a(af, kt, 0);
    read_b(b0, kt, 0);
    dma_b(1, kt + 1);
    bar();
    lgkm0();
    mma(af, b0, 0, 0);
    bar();
    // P2
    read_b(b1, kt, 1);
    dma_a(1, kt + 1);
    vm_wait<2 * LA + 2 * LB>();
    bar();
    lgkm0();
    mma(af, b1, 0, 1);
    bar();
    // P3
    read_a(af, kt, 1);
    dma_a(0, kt + 2);
    bar();
    lgkm0();
    mma(af, b1, 1, 1);
    bar();
    // P4
    dma_b(0, kt + 2);
    vm_wait<2 * LA + LB>();
    bar();
    mma(af, b0, 1, 0);
    bar();
  }
  } else {
  // Two phases per K-tile (half the barriers; 32 MFMAs per cluster):
  //   S1 read A-top, B-left, B-right (t)   DMA bottom (t+1)              MFMA top x {left, right}
  //   S3 read A-bottom (t)                 DMA top, left, right (t+2)    MFMA bottom x {right, left}
  // With the wave groups one barrier apart, a piece is read by the LEADING group one barrier after the
  // lagging group passes the barrier that ends its own phase, so both the DMA retirement (vmcnt) and the
  // phase's own reads (lgkmcnt) are waited BEFORE the phase's first barrier: every wave's DMA of a piece
  // has landed before any wave reads it, and every wave's reads of a half have returned before any wave
  // restages it.  (Round 3's first form waited vmcnt after the MFMA cluster, one barrier too late for
  // the leading group: wrong tiles on busy chips -- rel. error 0.17 on the 256x128 tile at 8192 x 4096 x
  // 4096, tests/test_gemm_k64_gpu.py.)  Each wait leaves 2LA + 2LB pieces in flight.
  dma_a(0, 0);
  dma_b(0, 0);
  dma_b(1, 0);
  dma_a(1, 0);
  dma_a(0, 1);
  dma_b(0, 1);
  dma_b(1, 1);
  vm_wait<2 * LA + LB2>();
  bar();
  if constexpr (STAG) {
    if (lag) bar();
  }
#ifdef DTA_K64_TIMELINE
  K64_TL(1, k64_rt());
#endif
#ifdef DTA_K64_STAMP
  unsigned long long seg[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_prev = stamp_now();
#endif
  // DIM (DTA_K64_DMA_IN_MFMA): a phase's DMA pieces go out between the MFMAs of its cluster, after the
  // phase's first barrier -- later than the read-phase placement, so every restaged half was retired by
  // every wave's reads even earlier than that form guarantees; the waits then leave one phase's pieces
  // fewer in flight (S1: the previous S3's top / left / right; S3: the S1 bottom), three barrier
  // intervals after issue as before
  constexpr bool DIM = DTA_K64_DMA_IN_MFMA != 0;
  auto piece_a = [&](int h, int kt, int j) {
    const int ks = kofs + min(kt, nk - 1);
    if constexpr (BUF) bglds16(rsA, voA[h][j], (unsigned)(ks * stepA * 2), lds0 + aoff(h, kt & 1) + (j * NW + wave) * 1024);
    else glds16(srcA[h][j] + ks * stepA, lds + aoff(h, kt & 1) + (j * NW + wave) * 1024);
  };
  auto piece_b = [&](int h, int kt, int j) {
    const int ks = kofs + min(kt, nk - 1);
    if constexpr (BUF) bglds16(rsB, voB[BJ ? 0 : h][j], (unsigned)(ks * stepB * 2), lds0 + boff(h, kt & 1) + (j * NW + wave) * 1024);
    else glds16(srcB[BJ ? 0 : h][j] + ks * stepB, lds + boff(h, kt & 1) + (j * NW + wave) * 1024);
  };
  // the 2 x (2 NTH MTH) MFMAs of mma(af, bx, mh, nhx) then mma(af, by, mh, nhy), with piece p of NP issued
  // after MFMA (p + 1) * NM / (NP + 1)
  auto mma2_dma = [&](const bf16x8 (&bx)[NTH][2], int nhx, const bf16x8 (&by)[NTH][2], int nhy, int mh, auto issue,
                      auto NPc) __attribute__((always_inline)) {
    constexpr int NP = decltype(NPc)::value, NM = 4 * NTH * MTH, STEP = NM / (NP + 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    k64_static_for<NM>([&](auto mc) {
      constexpr int m = decltype(mc)::value, half = m / (NM / 2), r = m % (NM / 2);
      constexpr int kk = r / (NTH * MTH), ii = (r / MTH) % NTH, jj = r % MTH;
      const bf16x8(&bf)[NTH][2] = half == 0 ? bx : by;
      const int nh = half == 0 ? nhx : nhy;
      acc[nh * NTH + ii][mh * MTH + jj] =
          __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ii][kk], af[jj][kk], acc[nh * NTH + ii][mh * MTH + jj], 0, 0, 0);
      if constexpr ((m + 1) % STEP == 0 && (m + 1) / STEP <= NP) {
        __builtin_amdgcn_sched_barrier(0);
        issue(std::integral_constant<int, (m + 1) / STEP - 1>{});
        __builtin_amdgcn_sched_barrier(0);
      }
    });
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
  // kt2: kt with its parity as a compile-time constant (P = 0 / 1), so (kt2 & 1) folds into immediates;
  // P = -1: runtime parity (every tile but the buffer-DMA 256 x 256 one)
  auto ktile = [&](const int kt, auto P) {
    const int kt2 = decltype(P)::value < 0 ? kt : ((kt & ~1) | decltype(P)::value);
    read_a(af, kt2, 0);
    read_b(b0, kt2, 0);
    read_b(b1, kt2, 1);
    if constexpr (!DIM) dma_a(1, kt2 + 1);
    K64_STAMP(0);
    lgkm0();
    vm_wait<DIM ? LA + LB2 : 2 * LA + LB2>();  // bottom (t)
    K64_STAMP(1);
    bar();
    K64_STAMP(2);
    if constexpr (DIM) {
      mma2_dma(b0, 0, b1, 1, 0, [&](auto pc) { piece_a(1, kt2 + 1, decltype(pc)::value); },
               std::integral_constant<int, LA>{});
    } else {
      mma(af, b0, 0, 0);
      mma(af, b1, 0, 1);
    }
    mma_cs(af, 0);
    K64_STAMP(3);
    bar();
    K64_STAMP(4);
    read_a(af, kt2, 1);
    if constexpr (!DIM) {
      dma_a(0, kt2 + 2);
      dma_b(0, kt2 + 2);
      dma_b(1, kt2 + 2);
    }
    K64_STAMP(5);
    lgkm0();
    vm_wait<DIM ? LA : 2 * LA + LB2>();  // top, left, right (t+1)
    K64_STAMP(6);
    bar();
    K64_STAMP(7);
    if constexpr (DIM) {
      mma2_dma(b1, 1, b0, 0, 1, [&](auto pc) {
        constexpr int p = decltype(pc)::value;
        if constexpr (p < LA) piece_a(0, kt2 + 2, p);
        else if constexpr (BJ) piece_b(0, kt2 + 2, p - LA);
        else piece_b((p - LA) / LB, kt2 + 2, (p - LA) % LB);
      }, std::integral_constant<int, LA + LB2>{});
    } else {
      mma(af, b1, 1, 1);
      mma(af, b0, 1, 0);
    }
    mma_cs(af, 1);
    K64_STAMP(8);
    bar();
    K64_STAMP(9);
  };
  if constexpr (ILV) {
    for (int kt = 0; kt < nk; kt += 2) {
      ktile(kt, std::integral_constant<int, 0>{});
      if (kt + 1 < nk) ktile(kt + 1, std::integral_constant<int, 1>{});
    }
  } else {
    for (int kt = 0; kt < nk; ++kt) ktile(kt, std::integral_constant<int, -1>{});
  }
#ifdef DTA_K64_STAMP
  if (lane == 0) {
    unsigned long long* o = g.stamps + ((int64_t)blockIdx.x * NW + wave) * 10;
#pragma unroll
    for (int i = 0; i < 10; ++i) o[i] = seg[i];
  }
#endif
  }
  vm_wait<0>();  // the tail's dummy DMAs land before the workgroup's LDS is released
#ifdef DTA_K64_TIMELINE
  K64_TL(2, k64_rt());
#endif
  if constexpr (STAG) {
    if (!lag) bar();  // equal barrier counts for both halves
  }
  if constexpr (SK) {
    if (nk != nk_all) {  // a cut tile: publish this part; the last contributor to arrive finishes the tile
      constexpr int NQ = 4 * NTH * MTH, NT = 64 * NW;  // f32x4 accumulators per lane, threads
      constexpr unsigned SLAB = (unsigned)BM * BN * 4;
      const int64_t u0 = (int64_t)t * nk_all;
      const int lo = (int)(u0 / sk->span), hi = (int)((u0 + nk_all - 1) / sk->span);
      auto slab = [&](int w, int sl) __attribute__((always_inline)) {
        return __builtin_amdgcn_make_buffer_rsrc(sk->ws + ((int64_t)w * 2 + sl) * (SLAB / 4), 0, SLAB, 0x00020000);
      };
      {
        const __amdgpu_buffer_rsrc_t own = slab(wsk, slot);
#pragma unroll
        for (int i = 0; i < 2 * NTH; ++i)
#pragma unroll
          for (int j = 0; j < 2 * MTH; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), own,
                                                   (unsigned)(((i * 2 * MTH + j) * NT + tid) * 16), 0, 16);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
      __syncthreads();
      int* flag = reinterpret_cast<int*>(lds);  // (the one LDS array: the K loop is done with it)
      if (tid == 0) {
        const int old = __hip_atomic_fetch_add(sk->cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == hi - lo;
        if (last) __hip_atomic_store(sk->cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
      }
      __syncthreads();
      const bool last = *flag != 0;
      __syncthreads();  // every wave has read the flag before the epilogue reuses the LDS
      if (!last) return;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (keeps the slab loads below the ticket)
      // the tile = the contributors' parts summed in K order, ((p_lo + ...) + p_hi), every part (this one too,
      // stored above) read back from its slab: the same bits whoever arrives last, one part of each fragment
      // row in flight at a time (the accumulators plus one row of parts fit the registers)
      auto slot_of = [&](int c) __attribute__((always_inline)) { return ((int64_t)c * sk->span) / nk_all == t ? 0 : 1; };
      for (int c = lo; c <= hi; ++c) {
        const __amdgpu_buffer_rsrc_t r = slab(c, slot_of(c));
#pragma unroll
        for (int i = 0; i < 2 * NTH; ++i) {
          f32x4 pa[2 * MTH];
#pragma unroll
          for (int j = 0; j < 2 * MTH; ++j)
            pa[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  r, (unsigned)(((i * 2 * MTH + j) * NT + tid) * 16), 0, 16));
#pragma unroll
          for (int j = 0; j < 2 * MTH; ++j) acc[i][j] = c == lo ? pa[j] : acc[i][j] + pa[j];
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      static_assert(NQ == 4 * NTH * MTH, "");
    }
  }

  if constexpr (CS) {
    if (do_cs && wc < MTH && (lane >> 4) == 0) {  // (the four columns of accb are equal)
#pragma unroll
      for (int h = 0; h < 2; ++h) g.db[m0 + h * HA + wr * (HA / WR) + 16 * wc + lane] = f2bf(accb[h][0]);
    }
  }
  // ---- epilogue: lane holds row m, columns n .. n+3 of each (i, j) fragment ----
  if constexpr (STG) {
    // tile image: row r at 2 BN r, its 16-B chunk c (CPR per row) at c ^ (r % CPR).  The residual /
    // GELU-input tile (EPI_RES / EPI_DGELU) comes into the same image first with whole-row loads (instead
    // of one 8-B read per lane per fragment), each lane replacing its four values by the result in place
    // (GPT-2 fc2 input gradient x gelu'(h): 78.1 -> 67.8 us).  The GELU dual store stages the rounded h and
    // computes gelu(h) from each row chunk as it leaves (one pass: through the LDS twice it measured 76.8 vs
    // 69.2 us per fragment, scripts/bench_fused_epi.py).
    // row bytes, chunks per row; each wave moves a contiguous run of the image's chunks, 64 per instruction
    // (whole rows for the power-of-two widths; CPR = 24 rows straddle instructions)
    constexpr int RB = 2 * BN, CPR = C::CPR, NIT = BM * CPR / (64 * NW);
    static_assert(BM * CPR % (64 * NW) == 0, "whole 64-chunk stores per wave");
    auto rowc = [&](int r, int& row, int& c) __attribute__((always_inline)) {
      const int q = wave * (BM * CPR / NW) + 64 * r + lane;
      row = q / CPR;
      c = q % CPR;
    };
    if constexpr (DSW) {
      // Two rounds through the tile image (it holds one bf16 tile): the a tile comes in with whole-row loads,
      // each lane turns its four values into db = g a s (in place) and keeps t = g s (1 + a (1 - s)) in its
      // accumulators; the db rows leave; then the b tile comes in and leaves as da = t b.  (The unfused path:
      // the product g stored, read back by swiglu_bwd_kernel with a and b, da / db written -- one [M, N] write
      // and read fewer here, and g is not rounded to bf16 first.)
      auto stage = [&](const bf16* src) {
#pragma unroll
        for (int r = 0; r < NIT; ++r) {
          int row, c;
          rowc(r, row, c);
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(src + (int64_t)(m0 + row) * g.ldr + n0 + 8 * c);
          *reinterpret_cast<bf16x8*>(lds + row * RB + 16 * (c ^ cswz<CPR>(row))) = v;
          if (r % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // (4 rows in flight: the t values stay live)
        }
        lgkm0();
        bar();
      };
      auto drain = [&](bf16* dst) {
        lgkm0();
        bar();
#pragma unroll
        for (int r = 0; r < NIT; ++r) {
          int row, c;
          rowc(r, row, c);
          *reinterpret_cast<bf16x8*>(dst + (int64_t)(m0 + row) * g.ldc + n0 + 8 * c) =
              *reinterpret_cast<const bf16x8*>(lds + row * RB + 16 * (c ^ cswz<CPR>(row)));
          if (r % 4 == 3) __builtin_amdgcn_sched_barrier(0);
        }
      };
      auto frag_px = [&](int i, int j) {
        const int nh = i / NTH, ii = i % NTH, mh = j / MTH, jj = j % MTH;
        const int nl = nh * HB + wc * (HB / WC) + 16 * ii + 4 * (lane >> 4);
        const int ml = mh * HA + wr * (HA / WR) + 16 * jj + (lane & 15);
        return reinterpret_cast<bf16x4*>(lds + ml * RB + 16 * ((nl >> 3) ^ cswz<CPR>(ml)) + 8 * ((nl >> 2) & 1));
      };
      const float al = alpha_of(g);
      bar();  // every wave's last fragment reads and DMA are done: the LDS is free
      stage(g.res);
#pragma unroll
      for (int i = 0; i < 2 * NTH; ++i)
#pragma unroll
        for (int j = 0; j < 2 * MTH; ++j) {
          bf16x4* px = frag_px(i, j);
          const bf16x4 a4 = *px;
          float db[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gv = acc[i][j][r] * al, a = bf2f(a4[r]);
            const float sg = 1.f / (1.f + __expf(-a));
            db[r] = gv * a * sg;
            acc[i][j][r] = gv * sg * (1.f + a * (1.f - sg));
          }
          *px = pk4_bf16(db[0], db[1], db[2], db[3]);
          __builtin_amdgcn_sched_barrier(0);  // one fragment at a time (hoisting every read costs registers)
        }
      drain(g.c + g.N);
      lgkm0();
      bar();  // every wave's image reads are done before the b tile overwrites it
      stage(g.res + g.N);
#pragma unroll
      for (int i = 0; i < 2 * NTH; ++i)
#pragma unroll
        for (int j = 0; j < 2 * MTH; ++j) {
          bf16x4* px = frag_px(i, j);
          const bf16x4 b4 = *px;
          *px = pk4_bf16(acc[i][j][0] * bf2f(b4[0]), acc[i][j][1] * bf2f(b4[1]), acc[i][j][2] * bf2f(b4[2]),
                         acc[i][j][3] * bf2f(b4[3]));
          __builtin_amdgcn_sched_barrier(0);
        }
      drain(g.c);
      return;
    }
    const bool has_res = g.epi == EPI_DGELU || g.epi == EPI_RES;
    const bool dual = g.epi == EPI_GELU && g.c2 != nullptr;
    bar();  // every wave's last fragment reads and DMA are done: the LDS is free
    if (has_res) {
#pragma unroll
      for (int r = 0; r < NIT; ++r) {
        int row, c;
        rowc(r, row, c);
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(g.res + (int64_t)(m0 + row) * g.ldr + n0 + 8 * c);
        *reinterpret_cast<bf16x8*>(lds + row * RB + 16 * (c ^ cswz<CPR>(row))) = v;
      }
      lgkm0();
      bar();
    }
#pragma unroll
    for (int i = 0; i < 2 * NTH; ++i) {
      const int nh = i / NTH, ii = i % NTH;
      const int nl = nh * HB + wc * (HB / WC) + 16 * ii + 4 * (lane >> 4);
      float bv[4];
      load_bias4(g, n0 + nl, bv);
#pragma unroll
      for (int j = 0; j < 2 * MTH; ++j) {
        const int mh = j / MTH, jj = j % MTH;
        const int ml = mh * HA + wr * (HA / WR) + 16 * jj + (lane & 15);
        bf16x4* px = reinterpret_cast<bf16x4*>(lds + ml * RB + 16 * ((nl >> 3) ^ cswz<CPR>(ml)) + 8 * ((nl >> 2) & 1));
        *px = has_res ? val4_res(g, acc[i][j], bv, *px) : val4(g, m0 + ml, n0 + nl, acc[i][j], bv, 0);
      }
    }
    lgkm0();
    bar();
#pragma unroll
    for (int r = 0; r < NIT; ++r) {
      int row, c;
      rowc(r, row, c);
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(lds + row * RB + 16 * (c ^ cswz<CPR>(row)));
#if defined(DTA_K64_EPI_DIAG) && DTA_K64_EPI_DIAG == 1
      if (g.alpha == -1234.5f)  // diagnostic build (scripts/k64_epi_diag.hip): stores skipped, values live
#endif
#if defined(DTA_K64_EPI_DIAG) && DTA_K64_EPI_DIAG == 2
      __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(g.c + (int64_t)(m0 + row) * g.ldc + n0 + 8 * c));
#else
      *reinterpret_cast<bf16x8*>(g.c + (int64_t)(m0 + row) * g.ldc + n0 + 8 * c) = v;
#endif
      if (dual) {
        const bf16x4 lo = pk4_bf16(gelu_fast(bf2f(v[0])), gelu_fast(bf2f(v[1])), gelu_fast(bf2f(v[2])), gelu_fast(bf2f(v[3])));
        const bf16x4 hi = pk4_bf16(gelu_fast(bf2f(v[4])), gelu_fast(bf2f(v[5])), gelu_fast(bf2f(v[6])), gelu_fast(bf2f(v[7])));
        *reinterpret_cast<bf16x8*>(g.c2 + (int64_t)(m0 + row) * g.ldc2 + n0 + 8 * c) =
            bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2 * NTH; ++i) {
    const int nh = i / NTH, ii = i % NTH;
    const int n = n0 + nh * HB + wc * (HB / WC) + 16 * ii + 4 * (lane >> 4);
    float bv[4];
    load_bias4(g, n, bv);
#pragma unroll
    for (int j = 0; j < 2 * MTH; ++j) {
      const int mh = j / MTH, jj = j % MTH;
      const int m = m0 + mh * HA + wr * (HA / WR) + 16 * jj + (lane & 15);
      store4(g, m, n, acc[i][j], bv);
    }
  }
}


template <int BM, int BN, int WC, bool AT, bool BT, int PH, bool BUF, bool STG = false, bool DSW = false, int WR = 2>
// (the 4-wave 128 x 192 tile held to 256 VGPRs: two workgroups per CU -- it took 272 otherwise)
__global__ void __launch_bounds__(64 * WR * WC, BN == 192 ? 2 : 1) gemm_k64_kernel(Args g) {
#ifdef DTA_K64_TIMELINE
  const unsigned long long t_entry = k64_rt();
#endif
  k64_body<BM, BN, WC, AT, BT, PH, BUF, false, STG, DSW, WR>(g, xcd_remap(blockIdx.x, g.tiles_m * g.tiles_n));
#ifdef DTA_K64_TIMELINE
  const unsigned long long t_issued = k64_rt();  // (the epilogue's stores issued, not yet drained)
  vm_wait<0>();
  const unsigned long long t_end = k64_rt();
  K64_TL(6, t_issued);
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  K64_TL(0, t_entry);
  K64_TL(3, t_end);
  K64_TL(4, (unsigned long long)hw);
  K64_TL(5, (unsigned long long)xcc);
#endif
}

// Stream-K form (SkArgs): workgroup w (XCD-remapped: consecutive runs share an XCD's L2) walks the units
// [w span, (w + 1) span) of the tile-major (tile, K-tile) order, one body call per tile segment
template <int BM, int BN, int WC, bool AT, bool BT, bool STG, int WR = 2>
__global__ void __launch_bounds__(64 * WR * WC, BN == 192 ? 2 : 1) gemm_k64_sk_kernel(Args g, SkArgs s) {
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int nk = g.K / BK;
  const int64_t units = (int64_t)g.tiles_m * g.tiles_n * nk;
  const int64_t u1 = min(units, (int64_t)(w + 1) * s.span);
  bool first = true;
  for (int64_t u = (int64_t)w * s.span; u < u1; first = false) {
    const int t = (int)(u / nk), kb = (int)(u - (int64_t)t * nk);
    const int ke = (int)min<int64_t>(nk, kb + (u1 - u));
    if (!first) __syncthreads();  // the previous segment's epilogue is done with the LDS
    k64_body<BM, BN, WC, AT, BT, 2, true, false, STG, false, WR, true>(g, t, kb, ke, &s, w, first ? 0 : 1);
    u += ke - kb;
  }
}

// Grouped weight gradients (on this kernel's 64-deep
// two-phase loop): dW_i = A_i^T B_i for several problems in ONE launch of 256 x 256 tiles over the
// full token reduction, the bias gradients from the same MFMA pipe (CS); the tiles of all problems
// form one list, XCD-remapped so each XCD takes a contiguous run.

template <bool BUF>
__global__ void __launch_bounds__(512) gemm_k64_group_kernel(GroupArgs ga) {
  const int t = xcd_remap(blockIdx.x, ga.tile_start[ga.n]);
  int q = 0;
  while (q + 1 < ga.n && t >= ga.tile_start[q + 1]) ++q;
  k64_body<256, 256, 4, true, true, 2, BUF, true, true>(ga.p[q], t - ga.tile_start[q]);
}

// stg: the staged epilogue (buffer DMA, one bf16 output)
template <int BM, int BN, int WC, bool AT, bool BT, bool BUF>
static hipError_t launch(const Args& g, int ph, bool stg, hipStream_t st) {
  if constexpr (BUF && !AT && BT) {  // EPI_DSWIGLU: the input-gradient layout, buffer DMA, staged, two-phase
    if (g.epi == EPI_DSWIGLU) {
      if (!stg || ph != 2) return hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_k64_kernel<BM, BN, WC, AT, BT, 2, BUF, true, true>), dim3(g.tiles_m * g.tiles_n),
                         dim3(128 * WC), 0, st, g);
      return hipGetLastError();
    }
  }
  if (g.epi == EPI_DSWIGLU) return hipErrorInvalidValue;
  if constexpr (BUF) {
    if (stg) {
      if (ph == 2)
        hipLaunchKernelGGL((gemm_k64_kernel<BM, BN, WC, AT, BT, 2, BUF, true>), dim3(g.tiles_m * g.tiles_n),
                           dim3(128 * WC), 0, st, g);
      else
        hipLaunchKernelGGL((gemm_k64_kernel<BM, BN, WC, AT, BT, 4, BUF, true>), dim3(g.tiles_m * g.tiles_n),
                           dim3(128 * WC), 0, st, g);
      return hipGetLastError();
    }
  }
  if (ph == 2)
    hipLaunchKernelGGL((gemm_k64_kernel<BM, BN, WC, AT, BT, 2, BUF>), dim3(g.tiles_m * g.tiles_n), dim3(128 * WC), 0, st,
                       g);
  else
    hipLaunchKernelGGL((gemm_k64_kernel<BM, BN, WC, AT, BT, 4, BUF>), dim3(g.tiles_m * g.tiles_n), dim3(128 * WC), 0, st,
                       g);
  return hipGetLastError();
}

template <int BM, int BN, int WC, bool BUF>
static hipError_t launch_l(const Args& g, bool at, bool bt, int ph, bool stg, hipStream_t st) {
  if (!at && !bt) return launch<BM, BN, WC, false, false, BUF>(g, ph, stg, st);
  if (!at && bt) return launch<BM, BN, WC, false, true, BUF>(g, ph, stg, st);
  if (at && bt) return launch<BM, BN, WC, true, true, BUF>(g, ph, stg, st);
  return launch<BM, BN, WC, true, false, BUF>(g, ph, stg, st);
}

// the 192-wide tiles (GPT-2's N = 768 / 2304 / 3072 / 50304 in whole tile columns): K-major A and B (the
// forward layout), two-phase loop, buffer-descriptor DMA only
template <int BM, int WC, int WR>
static hipError_t launch_192(const Args& g, bool at, bool bt, bool buf, bool stg, hipStream_t st) {
  if (at || bt || !buf || g.epi == EPI_DSWIGLU) return hipErrorInvalidValue;
  const dim3 grid(g.tiles_m * g.tiles_n), blk(64 * WR * WC);
  if (stg)
    hipLaunchKernelGGL((gemm_k64_kernel<BM, 192, WC, false, false, 2, true, true, false, WR>), grid, blk, 0, st, g);
  else
    hipLaunchKernelGGL((gemm_k64_kernel<BM, 192, WC, false, false, 2, true, false, false, WR>), grid, blk, 0, st, g);
  return hipGetLastError();
}

template <int BM, int BN, int WC, int WR = 2>
static hipError_t launch_sk(const Args& g, const SkArgs& s, int grid, bool at, bool bt, bool stg, hipStream_t st) {
  const dim3 gd(grid), blk(64 * WR * WC);
#define DTA_SK_L(AT_, BT_)                                                                                        \
  do {                                                                                                           \
    if (stg) hipLaunchKernelGGL((gemm_k64_sk_kernel<BM, BN, WC, AT_, BT_, true, WR>), gd, blk, 0, st, g, s);    \
    else hipLaunchKernelGGL((gemm_k64_sk_kernel<BM, BN, WC, AT_, BT_, false, WR>), gd, blk, 0, st, g, s);       \
  } while (0)
  if constexpr (BN == 192) {  // K-major operands only
    if (at || bt) return hipErrorInvalidValue;
    DTA_SK_L(false, false);
  } else {
    if (!at && !bt) DTA_SK_L(false, false);
    else if (!at && bt) DTA_SK_L(false, true);
    else if (at && bt) DTA_SK_L(true, true);
    else return hipErrorInvalidValue;  // (the TT layout: no stream-K instantiation)
  }
#undef DTA_SK_L
  return hipGetLastError();
}

template <int BM, int BN, int WC>
static hipError_t launch_t(const Args& g, bool at, bool bt, int ph, bool buf, bool stg, hipStream_t st) {
  return buf ? launch_l<BM, BN, WC, true>(g, at, bt, ph, stg, st) : launch_l<BM, BN, WC, false>(g, at, bt, ph, stg, st);
}

// tile ids: 1 = 256x256 (8 waves), 2 = 256x128 (8 waves), 3 = 128x128 (4 waves), 4 = 128x256 (8 waves);
// id + kTiles: the same tile with the two-phase K loop
constexpr int kTiles = 4;
// LDS-DMA form: buffer descriptors (bglds16) by default wherever every operand byte lies within 2 GiB
// of its base -- 1-5 % faster than flat global_load_lds at the GPT-2 / Llama shapes, never slower
// beyond noise (scripts/bench_k64buf.py, profiles/k64_buffer_dma.jsonl); tile-id bit kFlatDma forces
// the flat form (A/B), kBufDma is accepted for compatibility (= the default)
constexpr int kBufDma = 16;
// the 4-wave 256 x 256 tile with intra-wave read / MFMA overlap (csrc/gemm_w4.hip), every layout
constexpr int kW4 = 9;
constexpr int kW4S = 10;  // the same with the LDS-staged epilogue (whole 256-B row pieces per store)
constexpr int kFlatDma = 32;
constexpr int kNoStg = 128;  // tile-id bit: the per-fragment epilogue even where the staged one applies (A/B)
// 192-wide tiles (two-phase loop, K-major A and B only): 11 = 256 x 192 (8 waves, 4 x 2), 12 = 128 x 192
// (4 waves, 2 x 2; two workgroups per CU)
constexpr int kT192 = 11, kT192S = 12;
// tile-id bit: the stream-K form of a two-phase tile (5-8, 11, 12; buffer DMA), see SkArgs
constexpr int kSK = 64;
__host__ __device__ constexpr bool sk_base(int t) { return (t >= 5 && t <= 8) || t == kT192 || t == kT192S; }
// resident workgroups per CU of each two-phase tile (LDS: 128 / 96 / 64 / 96 / 112 / 80 KB; VGPRs)
__host__ __device__ constexpr int sk_per_cu(int t) { return t == 7 || t == kT192S ? 2 : 1; }
__host__ __device__ constexpr int tile_bm(int t) { return t == 3 || t == 4 || t == kT192S ? 128 : 256; }
__host__ __device__ constexpr int tile_bn(int t) { return t == kT192 || t == kT192S ? 192 : (t == 2 || t == 3 ? 128 : 256); }

}  // namespace k64
}  // namespace dta
