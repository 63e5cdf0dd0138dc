// W4: the 4-wave 256 x 256 bf16 GEMM tile with INTRA-wave read / MFMA overlap, NT layout
// (C[M, N] = alpha * A[M, K] B[N, K]^T (+ bias, epilogue)): the forward projections x W^T of the
// transformer blocks and the LM head -- SURVEY.md N07, nn.Linear at src/distributed_trainer.py:162,199
// scaled to the GPT-2 / Llama configs.  Dispatched as tile id 9 of csrc/gemm_k64.hip's entry point.
#include "gemm_epi.h"

#include <type_traits>

namespace dta {
namespace k64 {

// ------------------------------------------------------------------------------------------------
// W4: the 4-wave 256 x 256 tile with INTRA-wave read / MFMA overlap (NT: A [M][K], B [N][K] -- the
// forward projections x W^T and the LM head).  Round 3's 8-wave two-phase tile hid a wave's fragment
// reads behind its PARTNER's MFMAs, one barrier apart: 58.9 % MFMA busy and 38 % of the wave cycles
// parked in waits on the Llama o-projection (profiles/gemm_k64_vs_hipblaslt.txt).  Here each SIMD
// runs ONE wave that owns a 128 x 128 output (64 accumulators of 16 x 16, 256 AGPRs) and hides its
// own LDS reads and DMA issue between its own MFMAs:
//  * fragments double-buffered in registers at the 32-deep half-step (kk): while the 64 MFMAs of
//    half kk = 0 run, the 16 ds_read_b128 of half kk = 1 are issued between them (one per 4 MFMAs);
//    while half 1's MFMAs run, the 16 LDS-DMA pieces of K-tile t + 2 and then the 16 reads of K-tile
//    t + 1's half 0 are issued between them -- no lgkmcnt(0) between a read and unrelated MFMAs;
//  * two LDS images (64 KiB each, K-tile t in image t & 1), filled by buffer_load ... lds two K-tiles
//    ahead; TWO barriers per K-tile: B1 after the wave's last read of K-tile t (the image may be
//    refilled), B2 mid-way through half 1 after the counted vmcnt that retires K-tile t + 1's pieces
//    (its reads may start): the vmcnt is never 0 in the loop;
//  * rows of A / B past M / N are CLAMPED in the DMA source (the duplicated rows' accumulators are
//    never stored): 256-wide tiles cover N = 50304 (the GPT-2 head) with a predicated epilogue;
//  * the same XOR-swizzled K-major images and conflict-free ds_read_b128 fragment reads as above,
//    mfma(B, A) so a lane's four accumulators are four consecutive output columns.
// The structure is the one the library's best gfx950 kernel for these shapes uses (4 waves,
// 128 x 128 per wave, MI16x16, direct-to-LDS, prefetch depth 2 -- its kernel name and disassembly);
// the code is this file's own.
namespace w4 {
constexpr int IMG = 256 * BK * 2;                // one operand's K-tile image: 32 KiB
constexpr int LDS_BYTES = 4 * IMG;               // [A p0 | A p1 | B p0 | B p1]
constexpr int NP = IMG / 1024 / 4;               // 1 KiB DMA pieces per wave per operand per K-tile: 8
}  // namespace w4

__device__ __forceinline__ void w4_body(const Args& g, const int t) {
  __shared__ __attribute__((aligned(1024))) char lds[w4::LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;

  const int tiles_m = g.tiles_m, tiles_n = g.tiles_n;
  const int per_group = kGroupM * tiles_n;
  const int grp = t / per_group, in_g = t - grp * per_group;
  const int gm0 = grp * kGroupM, gh = min(kGroupM, tiles_m - gm0);
  const int m0 = (gm0 + in_g % gh) * 256, n0 = (in_g / gh) * 256;
  const int nk = g.K / BK;

  // ---- DMA: piece q (0..7) of this wave holds rows 32 q + 8 wave + (lane >> 3) of the tile, the lane's
  // 16-byte chunk XOR-swizzled by the row (row & 7 == lane >> 3); rows past M / N clamped ----
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.a), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.b), 0, 0x7fffffff, 0x00020000);
  unsigned voA[w4::NP], voB[w4::NP];
  {
    const int rl = 8 * wave + (lane >> 3), ch = (lane & 7) ^ (lane >> 3);
#pragma unroll
    for (int q = 0; q < w4::NP; ++q) {
      const int ra = min(m0 + 32 * q + rl, g.M - 1), rb = min(n0 + 32 * q + rl, g.N - 1);
      voA[q] = (unsigned)(((int64_t)ra * g.lda + 8 * ch) * 2);
      voB[q] = (unsigned)(((int64_t)rb * g.ldb + 8 * ch) * 2);
    }
  }
  const unsigned lds0 = lds_addr(lds);
  auto dma = [&](int kt, int par) {  // all 16 pieces of K-tile kt into image par (prologue form)
    const unsigned so = (unsigned)kt * (BK * 2);
#pragma unroll
    for (int q = 0; q < w4::NP; ++q) {
      bglds16(rsA, voA[q], so, lds0 + par * w4::IMG + (4 * q + wave) * 1024);
      bglds16(rsB, voB[q], so, lds0 + (2 + par) * w4::IMG + (4 * q + wave) * 1024);
    }
  };

  // ---- fragment reads: (row 16 j + (lane & 15) of the wave's 128-row half, k 32 kk + 8 (lane >> 4)) ----
  const int rrow = lane & 15, x = (lane >> 4) ^ (lane & 7);
  const int aoff[2] = {(wr * 128 + rrow) * 128 + 16 * x, (wr * 128 + rrow) * 128 + 16 * (x ^ 4)};
  const int boff[2] = {2 * w4::IMG + (wc * 128 + rrow) * 128 + 16 * x, 2 * w4::IMG + (wc * 128 + rrow) * 128 + 16 * (x ^ 4)};
  auto rd = [&](int off) { return *reinterpret_cast<const bf16x8*>(lds + off); };
  // The MFMA as inline asm with the accumulator pinned to AGPRs ("+a") and the fragments to VGPRs:
  // with the builtin the register allocator re-permuted the 256 accumulators and parked fragments in
  // AGPRs every iteration (~530 v_accvgpr moves per 256 MFMAs).  Hazards: a dependent MFMA chain on one
  // accumulator is interlocked by the hardware; the fragments' ds_read -> MFMA waits are inserted by the
  // compiler (it sees the asm's VGPR inputs); the accumulators are read only after the drain below.
  auto mma = [](f32x4& c, const bf16x8& b, const bf16x8& a) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a0[8], b0[8], a1[8], b1[8];  // half-step 0 / 1 fragments: A rows (j), B rows (i)

  // one K-tile kt (P = its parity = image): MFMAs of both half-steps; between them the reads of half 1,
  // the DMA of K-tile kt + 2 into this image (past the last K-tile: the last one again, never read -- the
  // wait counts stay static) and the reads of K-tile kt + 1's half 0 (after the last K-tile: that
  // never-read reload, equally harmless)
  auto ktile = [&](const int kt, auto P) {
    constexpr int p = decltype(P)::value;
    // half 0: 64 MFMAs on a0 / b0; between them the 16 reads of half 1 of this K-tile
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < 8) b1[s] = rd(boff[1] + p * w4::IMG + s * 2048);
      else a1[s - 8] = rd(aoff[1] + p * w4::IMG + (s - 8) * 2048);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = 4 * s + q, j = idx >> 3, i = idx & 7;
        mma(acc[i][j], b0[i], a0[j]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    lgkm0();  // this wave's reads of K-tile kt are done
    bar();    // B1: every wave's are -- image p may be refilled
    // half 1: 64 MFMAs on a1 / b1; the DMA of K-tile kt + 2 between the first 32, the reads of K-tile kt + 1's
    // half 0 between the last 32
    const unsigned so = (unsigned)min(kt + 2, nk - 1) * (BK * 2);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < 8) bglds16(rsA, voA[s], so, lds0 + p * w4::IMG + (4 * s + wave) * 1024);
      else bglds16(rsB, voB[s - 8], so, lds0 + (2 + p) * w4::IMG + (4 * (s - 8) + wave) * 1024);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int idx = 2 * s + q, j = idx >> 3, i = idx & 7;
        mma(acc[i][j], b1[i], a1[j]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    vm_wait<2 * w4::NP>();  // K-tile kt + 1 landed (this wave's pieces; kt + 2's stay in flight)
    bar();                  // B2: every wave's pieces of K-tile kt + 1 landed
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < 8) b0[s] = rd(boff[0] + (p ^ 1) * w4::IMG + s * 2048);
      else a0[s - 8] = rd(aoff[0] + (p ^ 1) * w4::IMG + (s - 8) * 2048);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int idx = 32 + 2 * s + q, j = idx >> 3, i = idx & 7;
        mma(acc[i][j], b1[i], a1[j]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- prologue: K-tiles 0 and 1 in flight, K-tile 0's half-0 fragments in registers ----
  dma(0, 0);
  dma(1, 1);
  vm_wait<2 * w4::NP>();
  bar();
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    b0[s] = rd(boff[0] + s * 2048);
    a0[s] = rd(aoff[0] + s * 2048);
  }
  // nk even (K % 128 == 0, checked on the host): pairs of K-tiles, parities compile-time constants, one
  // loop body and no tail -- branchy tails made the register allocator shuffle all 256 accumulators
  for (int kt = 0; kt < nk; kt += 2) {
    ktile(kt, std::integral_constant<int, 0>{});
    ktile(kt + 1, std::integral_constant<int, 1>{});
  }
  vm_wait<0>();  // the never-read reloads of the last iterations land before the LDS is released
  // the last MFMAs' results (in flight in the matrix pipe) before any v_accvgpr_read of the epilogue
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");

  // ---- epilogue: lane holds row m, columns n .. n+3 of each (i, j) fragment; rows / columns past M / N
  // (clamped duplicates) are not stored ----
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = n0 + wc * 128 + 16 * i + 4 * (lane >> 4);
    if (n >= g.N) continue;
    float bv[4];
    load_bias4(g, n, bv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = m0 + wr * 128 + 16 * j + (lane & 15);
      if (m < g.M) store4(g, m, n, acc[i][j], bv);
    }
  }
}

__global__ void __launch_bounds__(256, 1) gemm_w4_kernel(Args g) {
  w4_body(g, xcd_remap(blockIdx.x, g.tiles_m * g.tiles_n));
}

}  // namespace k64
}  // namespace dta

hipError_t dta_gemm_w4_launch(const dta::k64::Args& g, hipStream_t st) {
  hipLaunchKernelGGL(dta::k64::gemm_w4_kernel, dim3(g.tiles_m * g.tiles_n), dim3(256), 0, st, g);
  return hipGetLastError();
}
