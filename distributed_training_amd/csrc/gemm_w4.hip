// W4: the 4-wave 256 x 256 bf16 GEMM tile with INTRA-wave read / MFMA overlap, NT layout
// (C[M, N] = alpha * A[M, K] B[N, K]^T (+ bias, epilogue)): the forward projections x W^T of the
// transformer blocks and the LM head -- SURVEY.md N07, nn.Linear at src/distributed_trainer.py:162,199
// scaled to the GPT-2 / Llama configs.  Dispatched as tile ids 9 (per-fragment epilogue) / 10 (LDS-staged)
// of csrc/gemm_k64.hip's entry point; ops/lm.py times tile 10 against the k64 tiles and hipBLASLt per shape.
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
//    while half 1's MFMAs run, the 16 LDS-DMA pieces of K-tile t + 2 and the 16 reads of K-tile
//    t + 1's half 0 are issued between them -- no lgkmcnt(0) between a read and unrelated MFMAs;
//  * two LDS images (66 KiB each, K-tile t in image t & 1), filled by buffer_load ... lds two K-tiles
//    ahead, the pieces spread over the MFMAs (below); two barriers per K-tile: after the wave's last read
//    of an image (it may be refilled) and after the counted vmcnt that retires K-tile t + 1's pieces (its
//    reads may start): the vmcnt is never 0 in the loop;
//  * rows of A / B past M / N are CLAMPED in the DMA source (the duplicated rows' accumulators are
//    never stored): 256-wide tiles cover N = 50304 (the GPT-2 head) with a predicated epilogue;
//  * padded-piece K-major images (conflict-free ds_read_b128 fragment reads, in-order DMA sources),
//    mfma(B, A) so a lane's four accumulators are four consecutive output columns.
// The structure is the one the library's best gfx950 kernel for these shapes uses (4 waves,
// 128 x 128 per wave, MI16x16, direct-to-LDS, prefetch depth 2 -- its kernel name and disassembly);
// the code is this file's own.
namespace w4 {
constexpr int PIECE = 1056;                      // K-major 1 KiB DMA piece + 32 B of padding (see w4_body)
constexpr int IMG = 32 * PIECE;                  // one operand's K-tile image: 32 pieces (33 KiB)
constexpr int LDS_BYTES = 4 * IMG;               // [A p0 | A p1 | B p0 | B p1]
constexpr int NP = 8;                            // 1 KiB DMA pieces per wave per operand per K-tile
}  // namespace w4

// M/N-major image (transposed operand [K][M]): two 128-column halves of 64 k-rows x 256 B, chunk ch of
// k-row k stored at ch ^ mswz(k) (the conflict-free ds_read_b64_tr_b16 swizzle of gemm_k64.hip)
__device__ __forceinline__ int w4_mswz(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }

__device__ __forceinline__ bf16x4 w4_tr4(const char* lds, int byte_off) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(lds + byte_off));
  return __builtin_bit_cast(bf16x4, v);
}

// AT: A stored M-major [K][M] (weight gradients dy^T x); BT: B stored N-major [K][N] (input gradients dy W,
// weight gradients); otherwise K-major.  C = alpha A B^T in every case.
// KT: K is not a multiple of 128 (two K-tiles): the loop runs over ceil(K / 128) pairs and every DMA
// lane whose 8 k-values lie at or past K gets an out-of-range buffer offset -- the buffer unit returns
// zeros for it, so the tail contributes nothing (K a multiple of 8: chunks are whole).
// STG: LDS-staged epilogue (one bf16 output).
//
// K-major images (no per-lane swizzle: a DMA piece's lanes read whole 128-B row segments in order): piece p
// (0..31) holds rows p + 32 s (s = lane >> 3), lane & 7 = the 16-B chunk, at PIECE p -- row R at
// PIECE (R % 32) + 128 (R / 32).  The 32 B of padding per piece put the 16 rows an MFMA fragment read touches
// at 16-B units 2 (R % 8) + const: with the ds_read_b128 lane groups of MI355X_MICROARCH.md §LDS every group
// hits 16 distinct units -- conflict-free (checked by enumeration).  A fragment's reads at other j are
// immediate offsets.
//
// The K loop issues a wave's 16 DMA pieces of K-tile t + 2 among its 128 MFMAs of K-tile t after B1: A's 8
// between the first 32 MFMAs of half 1, B's 8 between the last 32 (one per 4 MFMAs; packed one per 2 MFMAs
// they cost ~55 issue cycles each -- profiles/gemm_w4_diagnostics.txt, with the schedules and the persistent
// form that were measured and dropped).
template <bool AT, bool BT, bool KT, bool STG>
__device__ __forceinline__ void w4_body(const Args& g, const int t, char* lds) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;

  const int tiles_m = g.tiles_m, tiles_n = g.tiles_n;
  const int per_group = kGroupM * tiles_n;
  const int grp = t / per_group, in_g = t - grp * per_group;
  const int gm0 = grp * kGroupM, gh = min(kGroupM, tiles_m - gm0);
  const int m0 = (gm0 + in_g % gh) * 256, n0 = (in_g / gh) * 256;
  const int nk = KT ? 2 * ((g.K + 2 * BK - 1) / (2 * BK)) : g.K / BK;

  // ---- DMA: this wave's 8 pieces per operand and K-tile, q = 0..7 ----
  // K-major: piece 4 q + wave.
  // M/N-major: piece gp = 4 q + wave holds k-rows 4 (gp & 15) + (lane >> 4) of column half gp >> 4, chunk
  //   (lane & 15) ^ mswz(k) (chunks past M / N clamped to the last full one); its half kk = (gp & 15) >= 8.
  // Rows past M / N are clamped to the last one (their accumulators are never stored).
  // (the base pointers through readfirstlane: the descriptor must live in SGPRs for the asm, and a kernel
  // grown by the staged epilogue lost the compiler's proof that g's fields are uniform)
  auto uni = [](const bf16* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<bf16*>(((uint64_t)hi << 32) | lo);
  };
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(uni(g.a), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(uni(g.b), 0, 0x7fffffff, 0x00020000);
  unsigned voA[w4::NP], voB[w4::NP];
  auto src_off = [&](bool tr, int x0, int X, int64_t ld, int q) -> unsigned {
    if (!tr) {
      const int r = min(x0 + 4 * q + wave + 32 * (lane >> 3), X - 1);
      return (unsigned)(((int64_t)r * ld + 8 * (lane & 7)) * 2);
    }
    const int gp = 4 * q + wave, k = 4 * (gp & 15) + (lane >> 4);
    const int col = min(x0 + 128 * (gp >> 4) + 8 * ((lane & 15) ^ w4_mswz(k)), X - 8);
    return (unsigned)(((int64_t)k * ld + col) * 2);
  };
#pragma unroll
  for (int q = 0; q < w4::NP; ++q) {
    voA[q] = src_off(AT, m0, g.M, g.lda, q);
    voB[q] = src_off(BT, n0, g.N, g.ldb, q);
  }
  // the k (within a K-tile) of this lane's 8 values in piece q
  auto lane_k = [&](bool tr, int q) {
    if (tr) return 4 * ((4 * q + wave) & 15) + (lane >> 4);
    return 8 * (lane & 7);
  };
  auto kt_off = [&](unsigned vo, bool tr, int q, int kt) -> unsigned {  // the K-tail's zero fill
    if constexpr (!KT) return vo;
    return kt * BK + lane_k(tr, q) < g.K ? vo : 0x80000000u;
  };
  const unsigned kstepA = AT ? (unsigned)(BK * g.lda * 2) : (unsigned)(BK * 2);
  const unsigned kstepB = BT ? (unsigned)(BK * g.ldb * 2) : (unsigned)(BK * 2);
  const unsigned lds0 = lds_addr(lds);
  // byte offset of this wave's piece q inside an operand image
  auto pdst = [&](bool tr, int q) -> unsigned {
    return (4 * q + wave) * (tr ? 1024 : w4::PIECE);
  };
  auto piece = [&](int op, int q, int kt, int par) {  // piece q of operand op (0 A, 1 B) of K-tile kt -> image par
    if (op == 0) bglds16_m0(rsA, kt_off(voA[q], AT, q, kt), (unsigned)kt * kstepA, lds0 + par * w4::IMG + pdst(AT, q));
    else bglds16_m0(rsB, kt_off(voB[q], BT, q, kt), (unsigned)kt * kstepB, lds0 + (2 + par) * w4::IMG + pdst(BT, q));
  };
  auto dma = [&](int kt, int par) {  // all 16 pieces of K-tile kt into image par (prologue form)
#pragma unroll
    for (int q = 0; q < w4::NP; ++q) {
      piece(0, q, kt, par);
      piece(1, q, kt, par);
    }
  };

  // ---- fragment reads: (index 16 j + (lane & 15) of the wave's 128-wide half, k 32 kk + 8 (lane >> 4)) ----
  // K-major: one ds_read_b128 at a per-lane base (per kk) + an immediate per j.  M/N-major: two
  // ds_read_b64_tr_b16 (k-rows 32 kk + 8 g + q and + 4, g = lane >> 4, q = (lane >> 2) & 3) at per-lane, per-j
  // offsets: the chunk 2 j + (p >> 1) (p = lane & 3) XOR the row swizzle is (j ^ c) * 32 + ..., c = 2 q + (g & 1).
  const int rrow = lane & 15;
  int kofA[2], kofB[2];                 // K-major per-kk lane bases
  int tlo[8], thi[8];                   // M/N-major per-j lane offsets inside a half image (lo / hi rows)
  {
    const int gg = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3, c = 2 * qq + (gg & 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      tlo[j] = (8 * gg + qq) * 256 + 32 * (j ^ c) + 16 * (pp >> 1) + 8 * (pp & 1);
      thi[j] = (8 * gg + qq + 4) * 256 + 32 * (j ^ c) + 16 * ((pp >> 1) ^ 1) + 8 * (pp & 1);
    }
  }
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    // R = 128 w + 16 j + rrow: PIECE (rrow + 16 (j & 1)) + 128 (4 w + (j >> 1)) + 16 (4 kk + (lane >> 4))
    const int base = w4::PIECE * rrow + 16 * (4 * kk + (lane >> 4));
    kofA[kk] = base + 512 * wr;
    kofB[kk] = base + 512 * wc;
  }
  const char* imgA = lds + (AT ? wr * 16384 : 0);  // M/N-major: two 16 KiB halves (pieces 0-15, 16-31)
  const char* imgB = lds + 2 * w4::IMG + (BT ? wc * 16384 : 0);
  auto frag = [&](bool tr, const char* img, const int (&kof)[2], int par, int kk, int j) -> bf16x8 {
    if (!tr) {
      const int jo = 16 * w4::PIECE * (j & 1) + 128 * (j >> 1);
      return *reinterpret_cast<const bf16x8*>(img + par * w4::IMG + kof[kk] + jo);
    }
    const char* b = img + par * w4::IMG + kk * 8192;
    const bf16x4 lo = w4_tr4(b, tlo[j]), hi = w4_tr4(b, thi[j]);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto rdA = [&](int par, int kk, int j) { return frag(AT, imgA, kofA, par, kk, j); };
  auto rdB = [&](int par, int kk, int j) { return frag(BT, imgB, kofB, par, kk, j); };
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
  // one K-tile kt (P = its parity = image): MFMAs of both half-steps; between them the reads of half 1, the
  // DMA of K-tile kt + 2 into this image (past the last K-tile: the last one again, never read -- the wait
  // counts stay static) and the reads of K-tile kt + 1's half 0 (after the last K-tile: that never-read reload)
  auto ktile = [&](const int kt, auto P) {
    constexpr int p = decltype(P)::value;
    const int kn = min(kt + 2, nk - 1);
    // half 0: 64 MFMAs on a0 / b0; between them the 16 reads of half 1 of this K-tile
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < 8) b1[s] = rdB(p, 1, s);
      else a1[s - 8] = rdA(p, 1, s - 8);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = 4 * s + q, j = idx >> 3, i = idx & 7;
        mma(acc[i][j], b0[i], a0[j]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    lgkm0();  // this wave's reads of K-tile kt are done
    bar();    // B1: every wave's are -- image p may be refilled
    // half 1: 64 MFMAs on a1 / b1; A's 8 pieces of K-tile kt + 2 between the first 32, the reads of K-tile
    // kt + 1's half 0 and B's 8 pieces between the last 32
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s % 2 == 0) piece(0, s / 2, kn, p);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int idx = 2 * s + q, j = idx >> 3, i = idx & 7;
        mma(acc[i][j], b1[i], a1[j]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    vm_wait<w4::NP>();  // B2: K-tile kt + 1 landed in every wave (K-tile kt + 2's 8 pieces of A stay in flight)
    bar();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < 8) b0[s] = rdB(p ^ 1, 0, s);
      else a0[s - 8] = rdA(p ^ 1, 0, s - 8);
      if (s % 2 == 0) piece(1, s / 2, kn, p);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int idx = 32 + 2 * s + q, j = idx >> 3, i = idx & 7;
        mma(acc[i][j], b1[i], a1[j]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // the zeroed accumulators pinned in AGPRs before the first MFMA (v_accvgpr_write -> MFMA SrcC needs
  // wait states the compiler cannot know to insert for an asm MFMA; the prologue's DMA issue and waits
  // below give far more)
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  // ---- prologue: K-tiles 0 and 1 in flight, K-tile 0's half-0 fragments in registers ----
  dma(0, 0);
  dma(1, 1);
  vm_wait<2 * w4::NP>();
  bar();
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    b0[s] = rdB(0, 0, s);
    a0[s] = rdA(0, 0, s);
  }
  // The last MFMAs' results are still in the matrix pipe when the loop ends: wait states before any
  // v_accvgpr_read.  The compiler does not know the asm statements are MFMAs, so every accumulator is then
  // passed through an empty asm ("+a") AFTER the nops -- volatile asm keeps its order, and the epilogue's
  // reads depend on those outputs.  (Without it hipcc read the last-written accumulators right behind their
  // MFMA: wrong sums in rows 240-255 of every tile, tests/test_gemm64_gpu.py.)
  auto drain = [&]() {
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  };
  // nk even (K % 128 == 0, or the K tail rounded up): pairs of K-tiles, parities compile-time constants, one
  // loop body and no tail -- branchy tails made the register allocator shuffle all 256 accumulators
  for (int kt = 0; kt < nk; kt += 2) {
    ktile(kt, std::integral_constant<int, 0>{});
    ktile(kt + 1, std::integral_constant<int, 1>{});
    // wait states behind the pair's last MFMAs: at the loop exit the register allocator may copy an
    // accumulator (v_accvgpr_read / _mov) before any statement of ours runs, and it does not know the asm
    // statements are MFMAs (24 cycles per 4096 MFMA cycles)
    asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
  }
  vm_wait<0>();  // the never-read reloads of the last iterations land before the LDS is released
  drain();
  // ---- epilogue: lane holds row m, columns n .. n+3 of each (i, j) fragment; rows / columns past M / N
  // (clamped duplicates) are not stored ----
  if constexpr (STG) {  // (the host takes this form only for one bf16 output: no c32, no GELU dual store)
    // LDS-staged: the wave's 128 x 128 bf16 result goes through its own 32 KiB of the (now free) LDS and
    // leaves as whole 256-B row pieces (one global_store_dwordx4 per lane: 4 rows per instruction)
    // instead of 64 stores of 16 rows x 32 B each.  Staging image: row r at 256 r, its 16-B chunk c at
    // c ^ (r & 15) (2-way conflicts at most on the 8-B writes, none on the row reads).
    bar();  // every wave's reads and DMA are done: the LDS is free
    char* st = lds + wave * (w4::IMG);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int nl = 16 * i + 4 * (lane >> 4);
      float bv[4];
      load_bias4(g, min(n0 + wc * 128 + nl, g.N - 4), bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ml = 16 * j + (lane & 15);
        const bf16x4 v = val4(g, min(m0 + wr * 128 + ml, g.M - 1), min(n0 + wc * 128 + nl, g.N - 4), acc[i][j], bv, 0);
        *reinterpret_cast<bf16x4*>(st + ml * 256 + 16 * ((nl >> 3) ^ (ml & 15)) + 8 * ((nl >> 2) & 1)) = v;
      }
    }
#pragma unroll
    for (int r = 0; r < 32; ++r) {
      const int row = 4 * r + (lane >> 4), c = lane & 15;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(st + row * 256 + 16 * (c ^ (row & 15)));
      const int m = m0 + wr * 128 + row, n = n0 + wc * 128 + 8 * c;
      if (m < g.M && n < g.N) *reinterpret_cast<bf16x8*>(g.c + (int64_t)m * g.ldc + n) = v;
    }
    return;
  }
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

template <bool AT, bool BT, bool KT, bool STG>
__global__ void __launch_bounds__(256, 1) gemm_w4_kernel(Args g) {
  __shared__ __attribute__((aligned(1024))) char lds[w4::LDS_BYTES];
  w4_body<AT, BT, KT, STG>(g, xcd_remap(blockIdx.x, g.tiles_m * g.tiles_n), lds);
}

// Grouped weight gradients (the contract of gemm_k64.hip's gemm_k64_group_kernel on the W4 pipeline, minus
// the bias gradient): dW_i = A_i^T B_i (A_i = dy [K][M_i], B_i = x [K][N_i]) for up to kGroupMax problems in
// one launch, the tiles of all problems one XCD-remapped list, LDS-staged stores.  Problems with a bias
// gradient go to the k64 group (ops/lm.py): W4 is chosen for the big bias-free Llama projections, and the
// extra db MFMAs pushed this kernel past the register file (the AGPRs hold the 256 accumulators).
template <bool KT>
__global__ void __launch_bounds__(256, 1) gemm_w4_group_kernel(GroupArgs ga) {
  // the problem's Args read in place from the kernel-argument segment (GroupArgs is the only argument,
  // at offset 0): indexing the by-value struct with the runtime q made the compiler copy all 16 Args
  const GroupArgs* gp = (const GroupArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  const int t = xcd_remap(blockIdx.x, gp->tile_start[gp->n]);
  int q = 0;
  while (q + 1 < gp->n && t >= gp->tile_start[q + 1]) ++q;
  q = __builtin_amdgcn_readfirstlane(q);
  __shared__ __attribute__((aligned(1024))) char lds[w4::LDS_BYTES];
  w4_body<true, true, KT, true>(gp->p[q], t - gp->tile_start[q], lds);
}

}  // namespace k64
}  // namespace dta

hipError_t dta_gemm_w4_wgrad_group(int n, const void* const* a, const int64_t* lda, const void* const* b,
                                   const int64_t* ldb, void* const* c, const int64_t* ldc, const int* M, const int* N,
                                   const int* K, void* const* db, hipStream_t st) {
  using namespace dta;
  using namespace dta::k64;
  if (n < 1 || n > kGroupMax) return hipErrorInvalidValue;
  GroupArgs ga{};
  ga.n = n;
  int total = 0;
  bool kt = false;
  for (int i = 0; i < n; ++i) {
    if (M[i] % 8 || N[i] % 8 || K[i] % 8 || K[i] < 8 || db[i] != nullptr) return hipErrorInvalidValue;
    if (2 * ((int64_t)(K[i] - 1) * lda[i] + M[i]) >= 0x7fffffffLL || 2 * ((int64_t)(K[i] - 1) * ldb[i] + N[i]) >= 0x7fffffffLL)
      return hipErrorInvalidValue;
    Args& g = ga.p[i];
    g.a = static_cast<const bf16*>(a[i]);
    g.b = static_cast<const bf16*>(b[i]);
    g.c = static_cast<bf16*>(c[i]);
    g.lda = lda[i];
    g.ldb = ldb[i];
    g.ldc = ldc[i];
    g.M = M[i];
    g.N = N[i];
    g.K = K[i];
    g.tiles_m = (M[i] + 255) / 256;
    g.tiles_n = (N[i] + 255) / 256;
    g.alpha = 1.f;
    g.epi = EPI_NONE;
    ga.tile_start[i] = total;
    total += g.tiles_m * g.tiles_n;
    kt = kt || K[i] % (2 * BK) != 0;
  }
  ga.tile_start[n] = total;
  if (kt) hipLaunchKernelGGL(gemm_w4_group_kernel<true>, dim3(total), dim3(256), 0, st, ga);
  else hipLaunchKernelGGL(gemm_w4_group_kernel<false>, dim3(total), dim3(256), 0, st, ga);
  return hipGetLastError();
}

template <bool KT, bool STG>
static void w4_launch(const dta::k64::Args& g, bool a_t, bool b_t, hipStream_t st) {
  using namespace dta::k64;
  const dim3 grid(g.tiles_m * g.tiles_n), block(256);
  if (!a_t && !b_t) hipLaunchKernelGGL((gemm_w4_kernel<false, false, KT, STG>), grid, block, 0, st, g);
  else if (!a_t && b_t) hipLaunchKernelGGL((gemm_w4_kernel<false, true, KT, STG>), grid, block, 0, st, g);
  else if (a_t && b_t) hipLaunchKernelGGL((gemm_w4_kernel<true, true, KT, STG>), grid, block, 0, st, g);
  else hipLaunchKernelGGL((gemm_w4_kernel<true, false, KT, STG>), grid, block, 0, st, g);
}

// staged: the LDS-staged epilogue (tile id 10) instead of per-fragment stores (tile id 9); one bf16 output only
// (no fp32 output, no GELU dual store: those take the per-fragment form)
hipError_t dta_gemm_w4_launch(const dta::k64::Args& g, bool a_t, bool b_t, bool staged_in, hipStream_t st) {
  using namespace dta::k64;
  const bool kt = g.K % (2 * BK) != 0;
  const bool one_out = g.c32 == nullptr && !(g.epi == EPI_GELU && g.c2 != nullptr);
  const bool staged = staged_in && one_out;
  if (kt) {
    if (staged) w4_launch<true, true>(g, a_t, b_t, st);
    else w4_launch<true, false>(g, a_t, b_t, st);
  } else {
    if (staged) w4_launch<false, true>(g, a_t, b_t, st);
    else w4_launch<false, false>(g, a_t, b_t, st);
  }
  return hipGetLastError();
}
