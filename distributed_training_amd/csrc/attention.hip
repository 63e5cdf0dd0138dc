// Flash attention forward / backward for gfx950 (MI355X), bf16 in, fp32 accumulate.
//
// Needed by the GPT-2 small and Llama-3 8B configurations of BASELINE.json
// (the reference itself has no attention: SURVEY.md §5.7).  Layout: tensors
// are [B, S, heads, D] with an arbitrary row (token) stride, so q/k/v can be
// read straight out of a fused QKV projection buffer and O is written ready for
// the output projection (no transposes).  GQA: q head h uses kv head
// h / (H / Hkv).  Causal or full.  D in {64, 128}.
//
// Every K/V/Q/dO tile is staged ONCE in LDS (the subtiled image of lo<D>
// below, conflict-free for all three access kinds) and read both by rows
// (ds_read_b128, MFMA operands whose k index is the head dim) and by columns
// with the gfx950 hardware-transpose read ds_read_b64_tr_b16 (operands whose
// k index is the key / query position).  Tiles are double-buffered in LDS and
// the next tile's global loads are issued into registers right after the
// single barrier of each step, so HBM latency hides behind the MFMAs.
//
// FORWARD (workgroup = 4 waves x 32 queries of one (batch, head)):
//   S^T = K . Q^T with the KEYS on the accumulator rows and the QUERIES on the
//   lanes, so the online-softmax max / sum are per-lane values (+ one lane^32
//   exchange); P stays in registers and is the B operand of O^T = V^T . P
//   (accumulator-as-operand, k order permuted; V^T fragments come from the
//   row-major V tile through transposed reads).
// BACKWARD, two atomic-free kernels (deterministic, no fp32 dQ buffer):
//   dK/dV (workgroup = 4 waves x 32 keys of one (batch, kv head)): keys on the
//     lanes, the workgroup's K/V staged once in LDS; per 64-query slice (all q
//     heads of the group) S = Q.K^T and dP = dO.V^T start from the row constants
//     -LSE/scale and -delta as initial accumulators, P = exp2(c S),
//     dS = P dP; dV^T += dO^T.P and dK^T += Q^T.dS take P / dS as the B
//     operand as they stand (dO^T / Q^T by transposed reads).
//   dQ (workgroup = 4 waves x 32 queries; runs FIRST): the forward's orientation;
//     delta = rowsum(dO * O) from its dO fragments and one read of O, stored for
//     dK/dV; S^T and dP^T recomputed per 64-key block, dQ^T += K^T . dS^T.
//   The 10 B H S^2 D FLOPs of a fused backward become 14 (S and dP are
//     computed twice) but the dQ float atomics -- bound at ~1.3 TB/s chip-wide
//     (MI355X_MICROARCH.md 'Global float atomics'), which dominated the fused
//     version at GPT-2 shapes -- disappear.
#include "common.h"
#include "attention.h"

#include <cstdlib>
#include <type_traits>

#ifndef DTA_DKDV_PF
#define DTA_DKDV_PF 3
#endif
#ifndef DTA_FWD_PF
#define DTA_FWD_PF 3
#endif
#ifndef DTA_DQ_PF
#define DTA_DQ_PF 3
#endif

namespace dta {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegBig = -1.0e30f;
// online-softmax rescale threshold (log2 domain): P up to 2^8 = 256 between rescales (bf16 / fp32 safe)
constexpr float kRescaleThr = 8.0f;

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// x[lane] (max | +) x[lane ^ 32] by v_permlane32_swap: a VALU op.  __shfl_xor goes through
// ds_bpermute, whose lgkmcnt(0) wait also waits for every fragment read the pipeline has in flight.
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// f(integral_constant<int, I>) for I = 0 .. N-1, unrolled at compile time (register-ring
// indices stay constants: a runtime index would put the ring in scratch)
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p supplies the address of
// row q (columns 4p..4p+3) of a 4 x 16 block; lane i receives column i of the
// four rows (row q in element q).
__device__ __forceinline__ bf16x4 lds_tr4(const bf16* p) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

// LDS images are unpadded [rows][D] bf16 tiles cut into 8-row x 32-column
// subtiles of 512 B (cdna_hip_programming.md T10, image (a)); inside a subtile
// row r holds its four 16-byte chunks in the order chunk ^ ((r >> 2) & 3).  All
// three accesses are conflict-free on this one image (scripts/lds_banks.py
// "subtiled", the lane-group / bank rules of MI355X_MICROARCH.md §LDS): the row
// read of an MFMA operand (ds_read_b128, lane = row, 16 B of the head dim), the
// transposed read (ds_read_b64_tr_b16, 4 rows x 16 columns per 16-lane group)
// and the register-staged 16-byte stores (tile_store's lane order).  Unlike a
// per-row XOR over all D / 8 chunks, the reads of one lane at other head-dim
// chunks / rows differ by a CONSTANT (+512 B per 32 columns, +D*16 B per 8
// rows): a fragment loop needs two base registers and immediate offsets, not
// one address register per k-step.  No padding keeps K+V double buffers at
// 32 KB (D = 64) / 64 KB (D = 128) per workgroup.
template <int D>
__device__ __forceinline__ int lo(int row, int col) {
  static_assert(D == 64 || D == 128, "head dim");
  const int ch = col >> 3;
  return (row >> 3) * (D * 8) + (ch >> 2) * 256 + (row & 7) * 32 + (((ch & 3) ^ ((row >> 2) & 3)) << 3) + (col & 7);
}

// A-operand fragment of X^T for a 32x32x16 MFMA whose B operand is an
// accumulator tile used as it stands (its row index is the k index, in the
// permuted order of cdna_hip_programming.md §3): lane (r32, hh) gets
// X[row0 + 16s + 8(j>>2) + 4hh + (j&3)][col0 + r32], j = 0..7, from the
// swizzled LDS image X by two transposed reads.
template <int D>
__device__ __forceinline__ bf16x8 tr_frag(const bf16* X, int row0, int col0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int r = row0 + 16 * s + 4 * (g >> 1) + (i >> 2);
  const int c = col0 + 16 * (g & 1) + 4 * (i & 3);
  const bf16x4 lo4 = lds_tr4(X + lo<D>(r, c));
  const bf16x4 hi4 = lds_tr4(X + lo<D>(r + 8, c));
  return bf16x8{lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
}

// MFMA row-operand fragment: row `row`, head-dim columns 16 ks + 8 hh .. + 7
template <int D>
__device__ __forceinline__ bf16x8 row_frag(const bf16* X, int row, int ks, int hh) {
  return *reinterpret_cast<const bf16x8*>(X + lo<D>(row, ks * 16 + hh * 8));
}

// Cooperative register staging of an [R][D] bf16 tile (NT threads, 16-byte
// loads), rows >= nrows zero-filled; then one store into the subtiled LDS image.
// Chunk e of the tile -> (row, column): a wave covers 8 rows x 128 B (whole
// 128-B lines of global memory), and each 8-lane group of its store covers two
// rows of one 512-B subtile = 128 contiguous LDS bytes (conflict-free
// ds_write_b128: MI355X_MICROARCH.md §LDS).
template <int D>
__device__ __forceinline__ void stage_rc(int e, int& r, int& c8) {
  constexpr int P = D / 64;  // 128-byte column pairs of chunk blocks per row
  const int l = e & 63, w = e >> 6;
  r = 8 * (w / P) + 2 * ((l >> 4) & 3) + ((l >> 2) & 1);
  c8 = 8 * (4 * (2 * (w % P) + ((l >> 3) & 1)) + (l & 3));
}

template <int R, int D, int NT>
struct TileRegs {
  static constexpr int N = R * D / 8 / NT;
  static_assert(N >= 1 && R * D == N * 8 * NT && R % 8 == 0 && NT % 64 == 0, "tile / thread count");
  bf16x8 v[N];
};

template <int R, int D, int NT>
__device__ __forceinline__ void tile_load(TileRegs<R, D, NT>& t, const bf16* base, int64_t rs, int row0, int nrows,
                                          int tid) {
#pragma unroll
  for (int l = 0; l < TileRegs<R, D, NT>::N; ++l) {
    int r, c8;
    stage_rc<D>(tid + l * NT, r, c8);
    if (row0 + r < nrows) {
      t.v[l] = *reinterpret_cast<const bf16x8*>(base + (int64_t)(row0 + r) * rs + c8);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) t.v[l][j] = f2bf(0.f);
    }
  }
}

template <int R, int D, int NT>
__device__ __forceinline__ void tile_store(const TileRegs<R, D, NT>& t, bf16* lds, int tid) {
#pragma unroll
  for (int l = 0; l < TileRegs<R, D, NT>::N; ++l) {
    int r, c8;
    stage_rc<D>(tid + l * NT, r, c8);
    *reinterpret_cast<bf16x8*>(lds + lo<D>(r, c8)) = t.v[l];
  }
}

// Buffer-descriptor form of tile_load: each thread's byte offsets within the tile are computed ONCE per
// kernel (tile_offsets) and a load is one buffer_load_dwordx4 at offset + the tile's first-row byte offset
// (one VALU add).  Rows past the matrix read as zeros through the descriptor's range check (num_records =
// the bytes up to the last row's D columns) -- instead of tile_load's per-load 64-bit address arithmetic
// and the exec-masked branch around every load (~150 instructions per 64-query slice of the dK/dV kernel,
// next to its 64 MFMAs at one wave per SIMD).  The host checks every such span is below 2 GiB.
template <int R, int D, int NT>
struct TileOffs {
  unsigned o[TileRegs<R, D, NT>::N];
};

template <int R, int D, int NT>
__device__ __forceinline__ void tile_offsets(TileOffs<R, D, NT>& t, int64_t rs, int tid) {
#pragma unroll
  for (int l = 0; l < TileRegs<R, D, NT>::N; ++l) {
    int r, c8;
    stage_rc<D>(tid + l * NT, r, c8);
    t.o[l] = (unsigned)((r * rs + c8) * 2);
  }
}

// descriptor over rows [0, nrows) of an [nrows][rs] bf16 matrix at `base` (D columns used per row)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const bf16* base, int64_t rs, int nrows, int D) {
  const uint64_t v = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  const int64_t bytes = nrows > 0 ? ((int64_t)(nrows - 1) * rs + D) * 2 : 0;
  const uint32_t num = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<bf16*>(((uint64_t)hi << 32) | lo), 0, num, 0x00020000);
}

template <int R, int D, int NT>
__device__ __forceinline__ void tile_load_buf(TileRegs<R, D, NT>& t, __amdgpu_buffer_rsrc_t rsrc,
                                              const TileOffs<R, D, NT>& o, unsigned row_bytes) {
#pragma unroll
  for (int l = 0; l < TileRegs<R, D, NT>::N; ++l) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o.o[l] + row_bytes, 0, 0);
    t.v[l] = __builtin_bit_cast(bf16x8, v);
  }
}

__device__ __forceinline__ f32x16 splat16(float x) {
  return f32x16{x, x, x, x, x, x, x, x, x, x, x, x, x, x, x, x};
}

// ------------------------------------------------------------------ forward
#ifndef DTA_FWD_RESCALE_BRANCH
#define DTA_FWD_RESCALE_BRANCH 1
#endif
// Online-softmax rescale of O and l when some row's max grew by more than kRescaleThr (log2 units):
// otherwise m stays and the block's P are bounded by 2^kRescaleThr (cdna_hip_programming.md T13; the
// decision precedes every exponentiation of the block, so nothing at the old max is left unscaled).
// The first block always rescales (m starts at -1e30).  DTA_FWD_RESCALE_BRANCH=0 (diagnostic builds,
// scripts/attn_diag.hip): no branch -- alpha = 1 on the common path, and no PHI copies of the O
// accumulators at the loop's back edge (the branchy form costs 32-64 v_mov_b64 per block at D = 128).
template <int NDT>
__device__ __forceinline__ void fwd_rescale(float mblk_c, float& m, float& l, f32x16 (&oacc)[NDT]) {
#if DTA_FWD_RESCALE_BRANCH
  if (__builtin_amdgcn_ballot_w64(mblk_c - m > kRescaleThr)) {
    const float mnew = fmaxf(m, mblk_c);
    const float alpha = fexp2(m - mnew);
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
    m = mnew;
  }
#else
  const bool up = __builtin_amdgcn_ballot_w64(mblk_c - m > kRescaleThr) != 0;
  const float mnew = up ? fmaxf(m, mblk_c) : m;
  const float alpha = fexp2(m - mnew);
  l *= alpha;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
  m = mnew;
#endif
}

// Occupancy the register budget is fitted to (waves per SIMD): the K/V double
// buffer is 32 KB (D = 64) / 64 KB (D = 128) per workgroup.
template <int D>
struct FwdCfg {
  static constexpr int kWavesPerSimd = D == 64 ? 3 : 2;
  static constexpr int kPrefetch = DTA_FWD_PF;  // D = 64 block compute
};

// Block id -> (query block, batch, head).  Under the causal mask the work of a
// query block grows with its index, so the heaviest blocks are dispatched
// first and the light ones fill the tail.  Consecutive ids walk the heads, so
// all query blocks of one head land on the same XCD (id % 8) whenever
// B * H % 8 == 0 and share its L2 copy of K / V.
__device__ __forceinline__ void fwd_block(int id, int BH, int nqb, bool causal, int& qb, int& bh) {
  bh = id % BH;
  qb = causal ? nqb - 1 - id / BH : id / BH;
}

template <int D, bool CAUSAL, int NW>
__global__ void __launch_bounds__(NW * 64, FwdCfg<D>::kWavesPerSimd) attn_fwd_kernel(AttnArgs a) {
  constexpr int NT = NW * 64;
  constexpr int QB = NW * 32;    // queries per workgroup
  constexpr int BN = 64;         // keys per block
  constexpr int NKS = D / 16;    // MFMA k-steps over D
  constexpr int NDT = D / 32;    // 32-wide output tiles over D
  __shared__ __attribute__((aligned(16))) bf16 Ks[2][BN * D];
  __shared__ __attribute__((aligned(16))) bf16 Vs[2][BN * D];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  int qb, bh;
  fwd_block(blockIdx.x, a.B * a.H, (a.S + QB - 1) / QB, CAUSAL, qb, bh);
  const int b = bh / a.H, h = bh % a.H;
  const int hk = h / (a.H / a.Hkv);
  const int q0w = qb * QB + wave * 32;
  const int qrow = q0w + r32;  // this lane's query row
  const bf16* qbase = static_cast<const bf16*>(a.q) + (int64_t)b * a.q_sb + (int64_t)h * D;
  const bf16* kbase = static_cast<const bf16*>(a.k) + (int64_t)b * a.k_sb + (int64_t)hk * D;
  const bf16* vbase = static_cast<const bf16*>(a.v) + (int64_t)b * a.v_sb + (int64_t)hk * D;

  // Q fragments (B operand of S^T = K.Q^T): lane (col q, half hh) holds Q[q][16ks + 8hh + j]
  bf16x8 qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (qrow < a.S)
      qf[ks] = *reinterpret_cast<const bf16x8*>(qbase + (int64_t)qrow * a.q_ss + ks * 16 + hh * 8);
    else
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = f2bf(0.f);
  }
  f32x16 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) oacc[dt] = splat16(0.f);
  float m = kNegBig, l = 0.f;   // running max (scaled, log2 domain) and sum
  const float c = a.scale * kLog2e;

  const int kv_end = CAUSAL ? min(qb * QB + QB, a.S) : a.S;
  const int nblk = (kv_end + BN - 1) / BN;
  // K / V tiles are register-staged (global -> registers -> swizzled LDS image).  D = 64:
  // TWO register sets, each tile loaded two blocks before its LDS store, so a load has
  // two blocks of compute to land in (one block -- ~1.5k cycles at D = 64 -- left the
  // loop waiting on vmcnt ~45 % of its wave-cycles: SQ_WAIT_ANY, profiles/pmc_attention_gpt2.txt);
  // the barrier after the store waits for LDS only (__syncthreads' fence would also wait
  // for the loads in flight).  D = 128: one set, one block ahead (register budget: the
  // loop below as it was).
  // One 64-key block against this wave's 32 queries (D = 64), software-pipelined like the
  // backward kernels: NS ops of S^T = K.Q^T (t = 32-key tile, k-step ks), the online softmax,
  // NP ops of O^T += V^T.P (t, 16-key half sh, 32-wide d tile dt); each op's LDS fragment is
  // read PF ops ahead into a register ring and sched_barriers pin the order.  (D = 128 keeps
  // the compiler's schedule below: at two waves per SIMD in 256 registers the ring spilled
  // and that forward ran 10-29 % slower.)
  auto attend = [&](const bf16* Kb, const bf16* Vb, int k0) __attribute__((always_inline)) {
    constexpr int NS = 2 * NKS, NP = 4 * NDT, TOT = NS + NP;
    constexpr int PF = FwdCfg<D>::kPrefetch, RING = PF + 1;
    bf16x8 ring[RING];
    f32x16 st[2];
    bf16x8 pb[2][2];
    auto issue = [&](auto oc) __attribute__((always_inline)) {
      constexpr int o = decltype(oc)::value;
      if constexpr (o < NS) {
        ring[o % RING] = row_frag<D>(Kb, (o / NKS) * 32 + r32, o % NKS, hh);
      } else {
        constexpr int cc = o - NS, t = cc / (2 * NDT), sh = (cc / NDT) % 2, dt = cc % NDT;
        ring[o % RING] = tr_frag<D>(Vb, t * 32, dt * 32, sh, lane);
      }
    };
    auto compute = [&](auto oc) __attribute__((always_inline)) {
      constexpr int o = decltype(oc)::value;
      if constexpr (o < NS) {
        constexpr int t = o / NKS, ks = o % NKS;
        if constexpr (ks == 0) st[t] = splat16(0.f);
        st[t] = mfma32x32x16(ring[o % RING], qf[ks], st[t]);
        if constexpr (o == NS - 1) {
          // ---- mask, online softmax (per-lane query row; scale folded into one FMA) ----
          const bool need_mask = (CAUSAL && k0 + BN - 1 > q0w) || k0 + BN > a.S;
          if (need_mask) {
            // key k0 + t*32 + row(i) + 4hh is masked past the sequence or (causal) past the
            // query: both are "block-relative row > lim", one compare against an immediate
            const int lim = min(a.S - 1, CAUSAL ? qrow : a.S) - k0 - 4 * hh;
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
              for (int i = 0; i < 16; ++i)
                if (t2 * 32 + mfma32_row(i, 0) > lim) st[t2][i] = kNegBig;
          }
          float mblk = st[0][0];
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
            for (int i = 0; i < 16; ++i) mblk = fmaxf(mblk, st[t2][i]);
          mblk = xor32_max(mblk);
          // rescale O and l only when some row's max grew by more than kRescaleThr (as below)
          fwd_rescale<NDT>(mblk * c, m, l, oacc);
          float lsum = 0.f;
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const float p = fexp2(__builtin_fmaf(st[t2][i], c, -m));
              st[t2][i] = p;
              lsum += p;
            }
          l += xor32_sum(lsum);
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
            for (int sh = 0; sh < 2; ++sh)
#pragma unroll
              for (int jj = 0; jj < 8; ++jj) pb[t2][sh][jj] = f2bf(st[t2][8 * sh + jj]);
        }
      } else {
        // ---- O^T += V^T . P  (V^T fragments by transposed reads of the V tile) ----
        constexpr int cc = o - NS, t = cc / (2 * NDT), sh = (cc / NDT) % 2, dt = cc % NDT;
        oacc[dt] = mfma32x32x16(ring[o % RING], pb[t][sh], oacc[dt]);
      }
    };
    static_for<PF>([&](auto oc) { issue(oc); });
    static_for<TOT>([&](auto oc) {
      constexpr int o = decltype(oc)::value;
      if constexpr (o + PF < TOT) issue(std::integral_constant<int, o + PF>{});
      __builtin_amdgcn_sched_barrier(0);
      compute(oc);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  const __amdgpu_buffer_rsrc_t rsK = rows_rsrc(kbase, a.k_ss, a.S, D), rsV = rows_rsrc(vbase, a.v_ss, a.S, D);
  TileOffs<BN, D, NT> offK, offV;
  tile_offsets(offK, a.k_ss, tid);
  tile_offsets(offV, a.v_ss, tid);
  auto kv_load = [&](TileRegs<BN, D, NT>& kr, TileRegs<BN, D, NT>& vr, int row0) __attribute__((always_inline)) {
    tile_load_buf(kr, rsK, offK, (unsigned)(row0 * a.k_ss * 2));
    tile_load_buf(vr, rsV, offV, (unsigned)(row0 * a.v_ss * 2));
  };
  if constexpr (D == 64) {
  constexpr int AHEAD = 2;
  TileRegs<BN, D, NT> krA, vrA, krB, vrB;
  kv_load(krA, vrA, 0);
  if (nblk > 1) kv_load(krB, vrB, BN);
  // (P: the block's LDS buffer parity, j & 1, as a compile-time constant: every LDS address of the block is a
  // lane base + an immediate, no per-block address arithmetic)
  auto block = [&](int j, TileRegs<BN, D, NT>& kr, TileRegs<BN, D, NT>& vr, auto P) __attribute__((always_inline)) {
    constexpr int buf = decltype(P)::value;
    tile_store(kr, Ks[buf], tid);
    tile_store(vr, Vs[buf], tid);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (j + AHEAD < nblk) kv_load(kr, vr, (j + AHEAD) * BN);  // its latency hides behind AHEAD blocks of MFMAs
      const int k0 = j * BN;
      if (CAUSAL && k0 > q0w + 31) return;  // every key of the block is after this wave's queries
      attend(Ks[buf], Vs[buf], k0);
  };
  for (int j = 0; j < nblk; j += 2) {
    block(j, krA, vrA, std::integral_constant<int, 0>{});
    if (j + 1 < nblk) block(j + 1, krB, vrB, std::integral_constant<int, 1>{});
  }
  } else {
    TileRegs<BN, D, NT> kr, vr;
    kv_load(kr, vr, 0);
    auto blk = [&](int j, auto P) __attribute__((always_inline)) {
      constexpr int buf = decltype(P)::value;  // (compile-time LDS buffer parity, as the D = 64 path)
      tile_store(kr, Ks[buf], tid);
      tile_store(vr, Vs[buf], tid);
      __syncthreads();
#if defined(DTA_ATTN_HOT_DIAG) && DTA_ATTN_HOT_DIAG
      if (j + 1 < nblk) kv_load(kr, vr, 0);  // diagnostic build only
#else
      if (j + 1 < nblk) kv_load(kr, vr, (j + 1) * BN);  // next tile's HBM latency hides behind this tile's MFMAs
#endif
      const int k0 = j * BN;
      if (CAUSAL && k0 > q0w + 31) return;  // every key of the block is after this wave's queries
      const bf16* Kb = Ks[buf];
      const bf16* Vb = Vs[buf];
      // ---- S^T tiles (raw scores): rows = keys k0 + t*32 + row, cols = this wave's queries ----
      f32x16 st[2];
  #pragma unroll
      for (int t = 0; t < 2; ++t) {
        st[t] = splat16(0.f);
  #pragma unroll
        for (int ks = 0; ks < NKS; ++ks) st[t] = mfma32x32x16(row_frag<D>(Kb, t * 32 + r32, ks, hh), qf[ks], st[t]);
      }
      // ---- mask, online softmax (per-lane query row; scale folded into one FMA) ----
      const bool need_mask = (CAUSAL && k0 + BN - 1 > q0w) || k0 + BN > a.S;
      if (need_mask) {
        const int lim = min(a.S - 1, CAUSAL ? qrow : a.S) - k0 - 4 * hh;  // as attend()
  #pragma unroll
        for (int t = 0; t < 2; ++t)
  #pragma unroll
          for (int i = 0; i < 16; ++i)
            if (t * 32 + mfma32_row(i, 0) > lim) st[t][i] = kNegBig;
      }
      float mblk = st[0][0];
  #pragma unroll
      for (int t = 0; t < 2; ++t)
  #pragma unroll
        for (int i = 0; i < 16; ++i) mblk = fmaxf(mblk, st[t][i]);
      mblk = xor32_max(mblk);
      // rescale O and l only when some row's max grew by more than kRescaleThr (log2 units):
      // otherwise m stays and this block's P are bounded by 2^kRescaleThr (cdna_hip_programming.md
      // T13; the decision precedes every exponentiation of the block, so nothing at the old max
      // is left unscaled).  The first block always rescales (m starts at -1e30).
      fwd_rescale<NDT>(mblk * c, m, l, oacc);
      float lsum = 0.f;
  #pragma unroll
      for (int t = 0; t < 2; ++t)
  #pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = fexp2(__builtin_fmaf(st[t][i], c, -m));
          st[t][i] = p;
          lsum += p;
        }
      l += xor32_sum(lsum);
      // ---- O^T += V^T . P  (V^T fragments by transposed reads of the V tile) ----
  #pragma unroll
      for (int t = 0; t < 2; ++t)
  #pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 pb;
  #pragma unroll
          for (int jj = 0; jj < 8; ++jj) pb[jj] = f2bf(st[t][8 * s + jj]);
  #pragma unroll
          for (int dt = 0; dt < NDT; ++dt) oacc[dt] = mfma32x32x16(tr_frag<D>(Vb, t * 32, dt * 32, s, lane), pb, oacc[dt]);
        }
    };
    for (int j = 0; j < nblk; j += 2) {
      blk(j, std::integral_constant<int, 0>{});
      if (j + 1 < nblk) blk(j + 1, std::integral_constant<int, 1>{});
    }
  }
  // ---- epilogue: O = O^T^T / l ; LSE ----
  if (qrow < a.S) {
    const float inv = 1.f / l;
    bf16* orow = static_cast<bf16*>(a.o) + (int64_t)b * a.o_sb + (int64_t)qrow * a.o_ss + (int64_t)h * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // rows 8g + 4hh + 0..3 are 4 consecutive d
        const bf16x4 ov = {f2bf(oacc[dt][4 * g] * inv), f2bf(oacc[dt][4 * g + 1] * inv),
                           f2bf(oacc[dt][4 * g + 2] * inv), f2bf(oacc[dt][4 * g + 3] * inv)};
        *reinterpret_cast<bf16x4*>(orow + dt * 32 + 8 * g + 4 * hh) = ov;
      }
    if (hh == 0) a.lse[((int64_t)b * a.H + h) * a.S + qrow] = (m + log2f(l)) / kLog2e;
  }
}

// ------------------------------------------------------------------ backward

// Query rows per slice of the dK/dV kernel: 64 (two 32-row MFMA tiles) halves
// the barriers per MFMA and doubles the compute behind each slice's prefetch
// (D = 128 runs one wave per SIMD: K/V fragments + dK/dV accumulators fill the
// register file; D = 64 keeps two; 32-row slices measured 5 % slower at GPT-2).
// Op order of a backward block of two 32-row tiles (ILV, the dK/dV slice and the dQ block): tile 0's NA
// score ops (S / dP) | tile 1's NA score ops + tile 0's softmax | tile 0's NC gradient ops + tile 1's softmax |
// tile 1's NC gradient ops.  op o -> (tile, op within the tile); without IL the tiles run one after the other.
template <bool IL, int NA, int NC>
__host__ __device__ constexpr int ilv_qt(int o) {
  return !IL ? o / (NA + NC) : (o < NA ? 0 : o < 2 * NA ? 1 : o < 2 * NA + NC ? 0 : 1);
}
template <bool IL, int NA, int NC>
__host__ __device__ constexpr int ilv_k(int o) {
  return !IL ? o % (NA + NC)
             : (o < NA ? o : o < 2 * NA ? o - NA : o < 2 * NA + NC ? NA + (o - 2 * NA) : NA + (o - 2 * NA - NC));
}
// the softmax part that op o carries (IL): {tile, part, elements per part} or tile -1 (none)
template <int NA, int NC>
__host__ __device__ constexpr int ilv_fill_tile(int o) {
  return o >= NA && o < 2 * NA ? 0 : o >= 2 * NA && o < 2 * NA + NC ? 1 : -1;
}
template <int NA, int NC>
__host__ __device__ constexpr int ilv_fill_part(int o) {
  return o < 2 * NA ? o - NA : o - 2 * NA;
}
template <int NA, int NC>
__host__ __device__ constexpr int ilv_fill_epp(int o) {
  return o < 2 * NA ? 16 / NA : 16 / NC;
}

// DTA_DKDV64_BM (diagnostic builds, scripts/attn_diag.hip): query rows per slice at D = 64 (32: three
// waves per SIMD fit the registers and three workgroups per CU the LDS)
#ifndef DTA_DKDV64_BM
#define DTA_DKDV64_BM 64
#endif
template <int D>
struct DkdvCfg {
  static constexpr int kBM = D == 64 ? DTA_DKDV64_BM : 64;
  static constexpr int kWavesPerSimd = D == 128 ? 1 : (kBM == 32 ? 3 : 2);
  static constexpr int kPrefetch = DTA_DKDV_PF;  // MFMA ops between a fragment's LDS read and its use
  static constexpr int kAhead = D == 64 && kBM == 64 ? 2 : 1;  // slices between a tile's global load and its LDS store
};

// The backward of rotate-half RoPE on one lane's accumulator row (row `pos`, d = dt * 32 + 8 g + 4 hh + j):
// the pairs (d, d + D/2) sit in tiles dt and dt + NDT/2 of the same lane -- dx1 = dy1 c + dy2 s,
// dx2 = dy2 c - dy1 s (rotation by -theta; lm_ops.hip rope_kernel with sign -1)
template <int D>
__device__ __forceinline__ void rope_inverse_acc(f32x16 (&acc)[D / 32], const float* rc, const float* rs, int pos,
                                                 int hh) {
  constexpr int NDT = D / 32, HALF = D / 2;
  const float* cr = rc + (int64_t)pos * HALF;
  const float* sr = rs + (int64_t)pos * HALF;
#pragma unroll
  for (int dt = 0; dt < NDT / 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int i0 = dt * 32 + 8 * g + 4 * hh;
      const float4 c4 = *reinterpret_cast<const float4*>(cr + i0);
      const float4 s4 = *reinterpret_cast<const float4*>(sr + i0);
      const float cv[4] = {c4.x, c4.y, c4.z, c4.w}, sv[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float y1 = acc[dt][4 * g + j], y2 = acc[dt + NDT / 2][4 * g + j];
        acc[dt][4 * g + j] = y1 * cv[j] + y2 * sv[j];
        acc[dt + NDT / 2][4 * g + j] = y2 * cv[j] - y1 * sv[j];
      }
    }
}

template <int D, bool CAUSAL, bool ILV>
__global__ void __launch_bounds__(256, DkdvCfg<D>::kWavesPerSimd) attn_bwd_dkdv_kernel(AttnArgs a) {
  constexpr int BM = DkdvCfg<D>::kBM;  // query rows per slice
  constexpr int NQT = BM / 32;         // 32-row query tiles per slice
  constexpr int NKS = D / 16;
  constexpr int NDT = D / 32;
  __shared__ __attribute__((aligned(16))) bf16 Qs[2][BM * D];
  __shared__ __attribute__((aligned(16))) bf16 dOs[2][BM * D];
  __shared__ __attribute__((aligned(16))) float rc[2][2][BM];  // [buf][-lse/scale | -delta][q] (16-B rows: float4 reads)
  // the workgroup's 128 keys of K and V, staged once: S / dP read their B operands from here
  // instead of keeping them in 64 (D = 128) registers, which pushed the working set past the
  // 256 arch VGPRs and made the compiler shuttle accumulators through AGPRs every slice
  __shared__ __attribute__((aligned(16))) bf16 KVs[2][128 * D];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  // key blocks in natural order = heaviest first under the causal mask;
  // consecutive ids walk (batch, kv head)
  const int BHk = a.B * a.Hkv;
  const int bk = blockIdx.x % BHk, b = bk / a.Hkv, hk = bk % a.Hkv;
  const int group = a.H / a.Hkv;
  const int kblk0 = (blockIdx.x / BHk) * 128;
  const int kw0 = kblk0 + wave * 32;  // this wave's first key
  const int key = kw0 + r32;          // this lane's key
  const bf16* kbase = static_cast<const bf16*>(a.k) + (int64_t)b * a.k_sb + (int64_t)hk * D;
  const bf16* vbase = static_cast<const bf16*>(a.v) + (int64_t)b * a.v_sb + (int64_t)hk * D;
  const float c = a.scale * kLog2e, inv_scale = 1.f / a.scale;

  {
    TileRegs<128, D, 256> kt, vt;  // (keys >= S zero-filled; visible after the loop's first barrier)
    tile_load(kt, kbase, a.k_ss, kblk0, a.S, tid);
    tile_load(vt, vbase, a.v_ss, kblk0, a.S, tid);
    tile_store(kt, KVs[0], tid);
    tile_store(vt, KVs[1], tid);
  }
  // D = 128 (one wave per SIMD): dK^T / dV^T accumulate in AGPRs through inline-asm MFMAs (this file's
  // MFMAs are otherwise in the VGPR
  // form): 128 (D = 128) fewer arch VGPRs, which is what lets the wave keep its 32 keys' K and V fragments
  // in registers below instead of re-reading them from LDS for every 32-query tile (a third of the
  // slice's LDS reads).  The compiler does not know the asm statements are MFMAs: the accumulators are
  // pinned through empty asm after wait states where they are written by VALU (the zeros) and before
  // they are read (the epilogue), as in csrc/gemm_w4.hip.
  f32x16 dvacc[NDT], dkacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dvacc[dt] = dkacc[dt] = splat16(0.f);
  constexpr bool KREG = D == 128;  // (D = 64 runs two waves per SIMD: its register budget keeps the LDS form)
  if constexpr (KREG) {
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) asm volatile("" : "+a"(dvacc[dt]), "+a"(dkacc[dt]));
  }
  auto mma_acc = [](f32x16& acc, const bf16x8& x, const bf16x8& y) {
    if constexpr (KREG) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(x), "v"(y));
    else acc = mfma32x32x16(x, y, acc);
  };
  bf16x8 kf[KREG ? NKS : 1], vf[KREG ? NKS : 1];  // this wave's 32 keys: B operands of S = Q.K^T, dP = dO.V^T
  if constexpr (KREG) {
    __syncthreads();  // the K / V tile images are complete
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      kf[ks] = row_frag<D>(KVs[0], wave * 32 + r32, ks, hh);
      vf[ks] = row_frag<D>(KVs[1], wave * 32 + r32, ks, hh);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  }

  const int qstart = CAUSAL ? kblk0 : 0;
  const int nslice = (a.S - qstart + BM - 1) / BM;
  const int total = nslice * group;
  // Q / dO tiles and the row constants of a slice are register-staged.  D = 64: TWO register
  // sets, each slice loaded two slices before its LDS store (one slice of MFMAs -- ~0.4 us --
  // does not cover the loads' latency; the forward's D = 64 path does the same), and the
  // barrier after the store waits for LDS only (__syncthreads' fence would also wait for the
  // other set's loads in flight).  D = 128: one set, one slice ahead (register budget).
  constexpr int AHEAD = DkdvCfg<D>::kAhead;
  struct Stage {
    TileRegs<BM, D, 256> q, d;
    float rc = 0.f;
  };
  Stage sA, sB;
  TileOffs<BM, D, 256> offQ, offD;  // (per-thread byte offsets, once: the slices only move the row offset)
  tile_offsets(offQ, a.q_ss, tid);
  tile_offsets(offD, a.do_ss, tid);
  auto load = [&](int it, Stage& st) __attribute__((always_inline)) {
    const int hq = hk * group + it / nslice;
#if defined(DTA_ATTN_HOT_DIAG) && DTA_ATTN_HOT_DIAG
    const int q0 = qstart;  // diagnostic build only (scripts/attn_diag.hip): every slice re-reads the first (L2-hot)
#else
    const int q0 = qstart + (it % nslice) * BM;
#endif
    tile_load_buf(st.q, rows_rsrc(static_cast<const bf16*>(a.q) + (int64_t)b * a.q_sb + (int64_t)hq * D, a.q_ss, a.S, D),
                  offQ, (unsigned)(q0 * a.q_ss * 2));
    tile_load_buf(st.d,
                  rows_rsrc(static_cast<const bf16*>(a.dout) + (int64_t)b * a.do_sb + (int64_t)hq * D, a.do_ss, a.S, D),
                  offD, (unsigned)(q0 * a.do_ss * 2));
    if (tid < 2 * BM) {
      const int qq = q0 + tid % BM;
      const int64_t ri = ((int64_t)b * a.H + hq) * a.S + qq;
      if (tid < BM) st.rc = qq < a.S ? -a.lse[ri] * inv_scale : kNegBig;  // q >= S: P = 0
      else st.rc = qq < a.S ? -a.delta[ri] : 0.f;
    }
  };
  load(0, sA);
  if (AHEAD == 2 && total > 1) load(1, sB);
  auto slice_it = [&](int it, Stage& cur, auto P) __attribute__((always_inline)) {
    constexpr int buf = decltype(P)::value;  // it & 1, compile-time: LDS addresses as immediates
    tile_store(cur.q, Qs[buf], tid);
    tile_store(cur.d, dOs[buf], tid);
    if (tid < 2 * BM) rc[buf][tid / BM][tid % BM] = cur.rc;
    if constexpr (AHEAD == 2) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else __syncthreads();
    if (it + AHEAD < total) load(it + AHEAD, cur);
    const int q0s = qstart + (it % nslice) * BM;
    if (CAUSAL && q0s + BM - 1 < kw0) return;  // all of this wave's keys are after the slice
    const bf16* Qb = Qs[buf];
    const bf16* Db = dOs[buf];
    // The slice as one software-pipelined stream of MFMA ops, per 32-query tile: NA ops of
    // S = Q.K^T - LSE/scale / dP = dO.V^T - delta (alternating), the softmax, then NC ops of
    // dV^T += dO^T.P / dK^T += Q^T.dS.  Every op's LDS fragments are read PF ops ahead into a
    // register ring and sched_barriers pin that order, so each MFMA waits on reads issued
    // PF MFMAs earlier (counted lgkmcnt) instead of on reads issued right before it -- the
    // compiler's own schedule put an lgkmcnt(0) before every MFMA of the D = 128 kernel.
    constexpr int NA = 2 * NKS, NC = 4 * NDT, NOP = NA + NC, TOT = NQT * NOP;
    constexpr int PF = DkdvCfg<D>::kPrefetch, RING = PF + 1;
    // ILV (two 32-query tiles, NA == NC): the op order tile-0 S/dP | tile-1 S/dP | tile-0 dV/dK | tile-1 dV/dK,
    // with tile 0's softmax spread over the tile-1 S/dP MFMAs and tile 1's over the tile-0 dV/dK MFMAs
    // (16 / NA score elements per MFMA gap: one exp2, two multiplies and half a bf16 pair-conversion each --
    // within the ~5 single-issue instructions a 32-cycle MFMA gap hides at one wave per SIMD,
    // MI355X_MICROARCH.md cycle constants; cdna_hip_programming.md T15).  Without it the softmax of a tile
    // sat between its S/dP and its dV/dK MFMAs with no MFMA in flight: ~130 VALU per tile, exposed.
    constexpr bool IL = ILV && NQT == 2 && 16 % NA == 0 && 16 % NC == 0;
    bf16x8 ring[RING][2];
    f32x16 s[NQT], dp[NQT];
    bf16x8 pb[NQT][2], db[NQT][2];
    auto issue = [&](auto oc) __attribute__((always_inline)) {
      constexpr int o = decltype(oc)::value, qt = ilv_qt<IL, NA, NC>(o), k = ilv_k<IL, NA, NC>(o);
      bf16x8(&f)[2] = ring[o % RING];
      if (k == 0) {
        // row constants of this lane's 16 accumulator rows as the initial accumulators: rows
        // qt*32 + 8g + 4hh + 0..3 are 4 consecutive floats
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int q4 = qt * 32 + 8 * g + 4 * hh;
          const float4 sv = *reinterpret_cast<const float4*>(&rc[buf][0][q4]);
          const float4 dv = *reinterpret_cast<const float4*>(&rc[buf][1][q4]);
          s[qt][4 * g] = sv.x; s[qt][4 * g + 1] = sv.y; s[qt][4 * g + 2] = sv.z; s[qt][4 * g + 3] = sv.w;
          dp[qt][4 * g] = dv.x; dp[qt][4 * g + 1] = dv.y; dp[qt][4 * g + 2] = dv.z; dp[qt][4 * g + 3] = dv.w;
        }
      }
      if constexpr (k < NA) {
        f[0] = row_frag<D>((k & 1) ? Db : Qb, qt * 32 + r32, k >> 1, hh);
        if constexpr (!KREG) f[1] = row_frag<D>(KVs[k & 1], wave * 32 + r32, k >> 1, hh);
      } else {
        constexpr int cc = k - NA, st = (cc >> 1) / NDT, dt = (cc >> 1) % NDT;
        f[0] = tr_frag<D>((cc & 1) ? Qb : Db, qt * 32, dt * 32, st, lane);
      }
    };
    // softmax of tile t, part j: score elements [j * E, (j + 1) * E) -> P = exp2(c S'), dS = P dP, and
    // their bf16 pairs (the B operands of the dV^T / dK^T MFMAs)
    auto sm_part = [&](auto tc, auto jc, auto ec) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value, j = decltype(jc)::value, E = decltype(ec)::value;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        constexpr int i0 = j * E;
        const int i = i0 + e;
        const float pv = fexp2(s[t][i] * c);
        s[t][i] = pv;              // P
        dp[t][i] = pv * dp[t][i];  // dS (unscaled)
        if (i & 1) {  // a finished pair -> packed bf16 (one v_cvt_pk each)
          pb[t][i >> 3][(i & 7) - 1] = f2bf(s[t][i - 1]);
          pb[t][i >> 3][i & 7] = f2bf(s[t][i]);
          db[t][i >> 3][(i & 7) - 1] = f2bf(dp[t][i - 1]);
          db[t][i >> 3][i & 7] = f2bf(dp[t][i]);
        }
        if constexpr (IL) {
          // pinned in this MFMA gap: the compiler would otherwise sink the whole softmax down to its first
          // use (the tile's dV / dK MFMAs), past the gaps it is meant to fill
          if (i & 1) asm volatile("" : "+v"(pb[t][i >> 3]), "+v"(db[t][i >> 3]));
          else asm volatile("" : "+v"(s[t][i]), "+v"(dp[t][i]));
        }
      }
      // pb / db are VALU results read by the asm MFMAs of the tile's dV / dK ops: wait states the compiler
      // cannot know to add
      if constexpr (KREG && (j + 1) * E == 16) asm volatile("s_nop 4" ::: "memory");
    };
    auto compute = [&](auto oc) __attribute__((always_inline)) {
      constexpr int o = decltype(oc)::value, qt = ilv_qt<IL, NA, NC>(o), k = ilv_k<IL, NA, NC>(o);
      const bf16x8(&f)[2] = ring[o % RING];
      if constexpr (k < NA) {
        if constexpr (KREG) {
          if (k & 1) dp[qt] = mfma32x32x16(f[0], vf[k >> 1], dp[qt]);
          else s[qt] = mfma32x32x16(f[0], kf[k >> 1], s[qt]);
        } else {
          if (k & 1) dp[qt] = mfma32x32x16(f[0], f[1], dp[qt]);
          else s[qt] = mfma32x32x16(f[0], f[1], s[qt]);
        }
        if constexpr (k == NA - 1) {
          // the causal mask of the tile as soon as its scores are complete (a wave-uniform branch: diagonal
          // tiles only), before any part of its softmax: key > query q0 + row(i) + 4hh <=> dl > row(i)
          const int q0 = q0s + qt * 32;
          if (CAUSAL && q0 < kw0 + 31) {
            const int dl = key - q0 - 4 * hh;
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if (dl > mfma32_row(i, 0)) s[qt][i] = kNegBig;  // exp2 -> P = 0
          }
          if constexpr (!IL)  // (the whole softmax of the tile right after its S / dP)
            sm_part(std::integral_constant<int, qt>{}, std::integral_constant<int, 0>{},
                    std::integral_constant<int, 16>{});
        }
      } else {
        constexpr int cc = k - NA, st = (cc >> 1) / NDT, dt = (cc >> 1) % NDT;
        if constexpr (cc & 1) mma_acc(dkacc[dt], f[0], db[qt][st]);
        else mma_acc(dvacc[dt], f[0], pb[qt][st]);
      }
      if constexpr (IL && ilv_fill_tile<NA, NC>(o) >= 0)
        sm_part(std::integral_constant<int, ilv_fill_tile<NA, NC>(o)>{},
                std::integral_constant<int, ilv_fill_part<NA, NC>(o)>{},
                std::integral_constant<int, ilv_fill_epp<NA, NC>(o)>{});
    };
    static_for<PF>([&](auto oc) { issue(oc); });
    static_for<TOT>([&](auto oc) {
      constexpr int o = decltype(oc)::value;
      if constexpr (o + PF < TOT) issue(std::integral_constant<int, o + PF>{});
      __builtin_amdgcn_sched_barrier(0);
      compute(oc);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  if constexpr (AHEAD == 2) {
    for (int it = 0; it < total; it += 2) {
      slice_it(it, sA, std::integral_constant<int, 0>{});
      if (it + 1 < total) slice_it(it + 1, sB, std::integral_constant<int, 1>{});
    }
  } else {
    for (int it = 0; it < total; it += 2) {
      slice_it(it, sA, std::integral_constant<int, 0>{});
      if (it + 1 < total) slice_it(it + 1, sA, std::integral_constant<int, 1>{});
    }
  }
  // the last MFMAs' results are still in the matrix pipe: wait states, then every accumulator through an
  // empty asm (the epilogue's reads depend on those outputs)
  if constexpr (KREG) {
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) asm volatile("" : "+a"(dvacc[dt]), "+a"(dkacc[dt]));
  }
  // ---- epilogue: dK = (dK^T)^T * scale, dV = (dV^T)^T ----
  if (key < a.S) {
    if (a.rcos) rope_inverse_acc<D>(dkacc, a.rcos, a.rsin, key, hh);
    bf16* dkr = static_cast<bf16*>(a.dk) + (int64_t)b * a.dk_sb + (int64_t)key * a.dk_ss + (int64_t)hk * D;
    bf16* dvr = static_cast<bf16*>(a.dv) + (int64_t)b * a.dv_sb + (int64_t)key * a.dv_ss + (int64_t)hk * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = dt * 32 + 8 * g + 4 * hh;
        const bf16x4 kv = {f2bf(dkacc[dt][4 * g] * a.scale), f2bf(dkacc[dt][4 * g + 1] * a.scale),
                           f2bf(dkacc[dt][4 * g + 2] * a.scale), f2bf(dkacc[dt][4 * g + 3] * a.scale)};
        const bf16x4 vv = {f2bf(dvacc[dt][4 * g]), f2bf(dvacc[dt][4 * g + 1]), f2bf(dvacc[dt][4 * g + 2]),
                           f2bf(dvacc[dt][4 * g + 3])};
        *reinterpret_cast<bf16x4*>(dkr + d0) = kv;
        *reinterpret_cast<bf16x4*>(dvr + d0) = vv;
      }
  }
}

// dQ keeps Q and dO fragments in registers: one wave per SIMD at D = 128.
template <int D>
struct DqCfg {
  static constexpr int kWavesPerSimd = D == 128 ? 1 : 2;
  static constexpr int kPrefetch = DTA_DQ_PF;
  static constexpr int kAhead = D == 64 ? 2 : 1;
};

template <int D, bool CAUSAL, int NW, bool ILV>
__global__ void __launch_bounds__(NW * 64, DqCfg<D>::kWavesPerSimd) attn_bwd_dq_kernel(AttnArgs a) {
  constexpr int NT = NW * 64;
  constexpr int QB = NW * 32;
  constexpr int BN = 64;
  constexpr int NKS = D / 16;
  constexpr int NDT = D / 32;
  __shared__ __attribute__((aligned(16))) bf16 Ks[2][BN * D];
  __shared__ __attribute__((aligned(16))) bf16 Vs[2][BN * D];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  int qb, bh;
  fwd_block(blockIdx.x, a.B * a.H, (a.S + QB - 1) / QB, CAUSAL, qb, bh);
  const int b = bh / a.H, h = bh % a.H;
  const int hk = h / (a.H / a.Hkv);
  const int q0w = qb * QB + wave * 32;
  const int qrow = q0w + r32;
  const bf16* qbase = static_cast<const bf16*>(a.q) + (int64_t)b * a.q_sb + (int64_t)h * D;
  const bf16* dobase = static_cast<const bf16*>(a.dout) + (int64_t)b * a.do_sb + (int64_t)h * D;
  const bf16* kbase = static_cast<const bf16*>(a.k) + (int64_t)b * a.k_sb + (int64_t)hk * D;
  const bf16* vbase = static_cast<const bf16*>(a.v) + (int64_t)b * a.v_sb + (int64_t)hk * D;
  const float c = a.scale * kLog2e;

  bf16x8 qf[NKS], df[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (qrow < a.S) {
      qf[ks] = *reinterpret_cast<const bf16x8*>(qbase + (int64_t)qrow * a.q_ss + ks * 16 + hh * 8);
      df[ks] = *reinterpret_cast<const bf16x8*>(dobase + (int64_t)qrow * a.do_ss + ks * 16 + hh * 8);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = df[ks][j] = f2bf(0.f);
    }
  }
  // delta = rowsum(dO * O) of this lane's query row, from the dO fragments already in registers
  // and the same fragments of O (each half-wave holds half the row: one lane^32 exchange); written
  // for the dK/dV kernel, which runs after this one (no separate delta pass)
  float dsum = 0.f;
  if (qrow < a.S) {
    const bf16* obase = static_cast<const bf16*>(a.o) + (int64_t)b * a.o_sb + (int64_t)qrow * a.o_ss + (int64_t)h * D;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(obase + ks * 16 + hh * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum += bf2f(ov[j]) * bf2f(df[ks][j]);
    }
  }
  dsum = xor32_sum(dsum);
  const int64_t ri = ((int64_t)b * a.H + h) * a.S + qrow;
  if (qrow < a.S && hh == 0) a.delta[ri] = dsum;
  // P = exp2(c S - c LSE / scale): the row constant rides in the exp's FMA (sb) and S^T starts from the MFMA's
  // inline-zero accumulator -- a splat of -LSE / scale into the 16 accumulators of both key tiles cost 32
  // v_mov per 64-key block at one wave per SIMD, where every non-MFMA instruction past ~5 per MFMA gap is
  // paid in full (MI355X_MICROARCH.md issue costs)
  const float sb = qrow < a.S ? -a.lse[ri] / a.scale * c : kNegBig;
  const float dp_init = qrow < a.S ? -dsum : 0.f;
  f32x16 dqacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dqacc[dt] = splat16(0.f);

  const int kv_end = CAUSAL ? min(qb * QB + QB, a.S) : a.S;
  const int nblk = (kv_end + BN - 1) / BN;
  // K / V register staging as the dK/dV kernel's Q / dO: two sets two blocks ahead at D = 64
  constexpr int AHEAD = DqCfg<D>::kAhead;
  struct Stage {
    TileRegs<BN, D, NT> k, v;
  };
  Stage sA, sB;
  const __amdgpu_buffer_rsrc_t rsK = rows_rsrc(kbase, a.k_ss, a.S, D), rsV = rows_rsrc(vbase, a.v_ss, a.S, D);
  TileOffs<BN, D, NT> offK, offV;
  tile_offsets(offK, a.k_ss, tid);
  tile_offsets(offV, a.v_ss, tid);
  auto kv_load = [&](Stage& st, int row0) __attribute__((always_inline)) {
    tile_load_buf(st.k, rsK, offK, (unsigned)(row0 * a.k_ss * 2));
    tile_load_buf(st.v, rsV, offV, (unsigned)(row0 * a.v_ss * 2));
  };
  kv_load(sA, 0);
  if (AHEAD == 2 && nblk > 1) kv_load(sB, BN);
  auto block_it = [&](int j, Stage& cur, auto P) __attribute__((always_inline)) {
    constexpr int buf = decltype(P)::value;  // j & 1, compile-time: LDS addresses as immediates
    tile_store(cur.k, Ks[buf], tid);
    tile_store(cur.v, Vs[buf], tid);
    if constexpr (AHEAD == 2) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else __syncthreads();
#if defined(DTA_ATTN_HOT_DIAG) && DTA_ATTN_HOT_DIAG
    if (j + AHEAD < nblk) kv_load(cur, 0);  // diagnostic build only: the first (L2-hot) block every time
#else
    if (j + AHEAD < nblk) kv_load(cur, (j + AHEAD) * BN);
#endif
    const int k0 = j * BN;
    if (CAUSAL && k0 > q0w + 31) return;
    const bf16* Kb = Ks[buf];
    const bf16* Vb = Vs[buf];
    const bool need_mask = CAUSAL && k0 + BN - 1 > q0w;
    // S^T = K.Q^T - LSE/scale, dP^T = V.dO^T - delta: rows = keys, cols = queries.
    // Keys >= S are zero rows of K and V: they add nothing to dQ.
    // Software-pipelined as the dK/dV slice: per 32-key tile NA ops of S^T / dP^T
    // (alternating), the softmax, NC ops of dQ^T += K^T . dS^T; each op's LDS fragment
    // is read PF ops ahead into a register ring (sched_barriers pin the order).
    constexpr int NA = 2 * NKS, NC = 2 * NDT, NOP = NA + NC, TOT = 2 * NOP;
    constexpr int PF = DqCfg<D>::kPrefetch, RING = PF + 1;
    // ILV: the dK/dV slice's op order (ilv_qt): tile 0's softmax in the tile-1 S^T / dP^T MFMA gaps, tile 1's
    // in the tile-0 dQ^T gaps, instead of a VALU block between a tile's score and gradient MFMAs
    constexpr bool IL = ILV && 16 % NA == 0 && 16 % NC == 0;
    bf16x8 ring[RING];
    f32x16 s[2], dp[2];
    bf16x8 db[2][2];
    auto issue = [&](auto oc) __attribute__((always_inline)) {
      constexpr int o = decltype(oc)::value, t = ilv_qt<IL, NA, NC>(o), k = ilv_k<IL, NA, NC>(o);
      if constexpr (k < NA) {
        ring[o % RING] = row_frag<D>((k & 1) ? Vb : Kb, t * 32 + r32, k >> 1, hh);
      } else {
        constexpr int cc = k - NA;
        ring[o % RING] = tr_frag<D>(Kb, t * 32, (cc % NDT) * 32, cc / NDT, lane);
      }
    };
    // softmax of tile t, part j (elements [j E, (j + 1) E)): dS^T = exp2(c S'^T) dP'^T and its bf16 pairs
    auto sm_part = [&](auto tc, auto jc, auto ec) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value, j = decltype(jc)::value, E = decltype(ec)::value;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = j * E + e;
        dp[t][i] *= fexp2(fmaf(s[t][i], c, sb));  // dS^T
        if (i & 1) {
          db[t][i >> 3][(i & 7) - 1] = f2bf(dp[t][i - 1]);
          db[t][i >> 3][i & 7] = f2bf(dp[t][i]);
          if constexpr (IL) asm volatile("" : "+v"(db[t][i >> 3]));  // pinned in this gap (see the dK/dV slice)
        } else if constexpr (IL) {
          asm volatile("" : "+v"(dp[t][i]));
        }
      }
    };
    auto compute = [&](auto oc) __attribute__((always_inline)) {
      constexpr int o = decltype(oc)::value, t = ilv_qt<IL, NA, NC>(o), k = ilv_k<IL, NA, NC>(o);
      const bf16x8& f = ring[o % RING];
      if constexpr (k < NA) {
        if constexpr (k == 0) {
          s[t] = splat16(0.f);
          dp[t] = splat16(dp_init);
        }
        if constexpr (k & 1) dp[t] = mfma32x32x16(f, df[k >> 1], dp[t]);
        else s[t] = mfma32x32x16(f, qf[k >> 1], s[t]);
        if constexpr (k == NA - 1) {
          // key k0 + t*32 + row(i) + 4hh > qrow <=> row(i) > ql
          if (need_mask) {  // wave-uniform: the diagonal blocks only
            const int ql = qrow - k0 - t * 32 - 4 * hh;
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if (mfma32_row(i, 0) > ql) s[t][i] = kNegBig;  // exp2 -> P = 0
          }
          if constexpr (!IL)
            sm_part(std::integral_constant<int, t>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, 16>{});
        }
      } else {
        constexpr int cc = k - NA;
        dqacc[cc % NDT] = mfma32x32x16(f, db[t][cc / NDT], dqacc[cc % NDT]);
      }
      if constexpr (IL && ilv_fill_tile<NA, NC>(o) >= 0)
        sm_part(std::integral_constant<int, ilv_fill_tile<NA, NC>(o)>{},
                std::integral_constant<int, ilv_fill_part<NA, NC>(o)>{},
                std::integral_constant<int, ilv_fill_epp<NA, NC>(o)>{});
    };
    static_for<PF>([&](auto oc) { issue(oc); });
    static_for<TOT>([&](auto oc) {
      constexpr int o = decltype(oc)::value;
      if constexpr (o + PF < TOT) issue(std::integral_constant<int, o + PF>{});
      __builtin_amdgcn_sched_barrier(0);
      compute(oc);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  if constexpr (AHEAD == 2) {
    for (int j = 0; j < nblk; j += 2) {
      block_it(j, sA, std::integral_constant<int, 0>{});
      if (j + 1 < nblk) block_it(j + 1, sB, std::integral_constant<int, 1>{});
    }
  } else {
    for (int j = 0; j < nblk; j += 2) {
      block_it(j, sA, std::integral_constant<int, 0>{});
      if (j + 1 < nblk) block_it(j + 1, sA, std::integral_constant<int, 1>{});
    }
  }
  if (qrow < a.S) {
    if (a.rcos) rope_inverse_acc<D>(dqacc, a.rcos, a.rsin, qrow, hh);
    bf16* dqr = static_cast<bf16*>(a.dq) + (int64_t)b * a.dq_sb + (int64_t)qrow * a.dq_ss + (int64_t)h * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const bf16x4 qv = {f2bf(dqacc[dt][4 * g] * a.scale), f2bf(dqacc[dt][4 * g + 1] * a.scale),
                           f2bf(dqacc[dt][4 * g + 2] * a.scale), f2bf(dqacc[dt][4 * g + 3] * a.scale)};
        *reinterpret_cast<bf16x4*>(dqr + dt * 32 + 8 * g + 4 * hh) = qv;
      }
  }
}

}  // namespace dta

using namespace dta;

// 8 waves (256 queries) per workgroup share each K/V tile when the grid still
// fills the chip several times over; 4 waves otherwise (GPT-2: S = 1024).
template <int D, int NW>
static void fwd_launch(const AttnArgs& a, bool causal, hipStream_t st) {
  const int nqb = (a.S + NW * 32 - 1) / (NW * 32);
  dim3 grid((unsigned)(nqb * a.B * a.H));
  if (causal) hipLaunchKernelGGL((attn_fwd_kernel<D, true, NW>), grid, dim3(NW * 64), 0, st, a);
  else hipLaunchKernelGGL((attn_fwd_kernel<D, false, NW>), grid, dim3(NW * 64), 0, st, a);
}

// 8 waves (256 queries) per workgroup share each K/V tile: measured faster
// whenever the grid still holds >= 1024 such workgroups (D = 128; Llama-3 8B shape 552 -> 526 us).
// At D = 64 the 8-wave form was faster at GPT-2's 384 workgroups before the forward's software
// pipeline (round 2: 43.6 -> 37.4 us); at HEAD the 4-wave form is (26.2-27.6 -> 24.3-24.8 us,
// profiles/attn_forms_r6k.jsonl), so both head dims take the same threshold.
static int fwd_waves(const AttnArgs& a, int D) {
  const char* force = getenv("DTA_ATTN_FWD_WAVES");  // tests / sweeps: "4" or "8"
  if (force) return atoi(force) == 8 ? 8 : 4;
  (void)D;
  const int64_t wg8 = (int64_t)((a.S + 255) / 256) * a.B * a.H;
  return wg8 >= 1024 ? 8 : 4;
}

static int dq_waves(const AttnArgs& a, int D) {
  const char* force = getenv("DTA_ATTN_DQ_WAVES");
  if (force) return atoi(force) == 8 ? 8 : 4;
  (void)a;
  (void)D;
  return 4;
}

template <int D>
static hipError_t fwd_d(const AttnArgs& a, bool causal, hipStream_t st) {
  if (fwd_waves(a, D) == 8) fwd_launch<D, 8>(a, causal, st);
  else fwd_launch<D, 4>(a, causal, st);
  return hipGetLastError();
}

// the backward kernels' interleaved softmax (ILV): the default at D = 128 (Llama-3 shape backward 1916-1954
// -> 1898-1944 us), not at D = 64 (GPT-2 shape 72.9 -> 76.4 us: its kernels have the registers and waves to
// hide the softmax already; profiles/attn_diag_r5e.jsonl).  DTA_ATTN_BWD_ILV=0 / 1 forces either (A/B).
static bool bwd_ilv(int D) {
  const char* e = getenv("DTA_ATTN_BWD_ILV");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return D == 128;
}

template <int D, int NW>
static void dq_launch(const AttnArgs& a, bool causal, hipStream_t st) {
  const int nqb = (a.S + NW * 32 - 1) / (NW * 32);
  dim3 grid((unsigned)(nqb * a.B * a.H));
  if (bwd_ilv(D)) {
    if (causal) hipLaunchKernelGGL((attn_bwd_dq_kernel<D, true, NW, true>), grid, dim3(NW * 64), 0, st, a);
    else hipLaunchKernelGGL((attn_bwd_dq_kernel<D, false, NW, true>), grid, dim3(NW * 64), 0, st, a);
  } else {
    if (causal) hipLaunchKernelGGL((attn_bwd_dq_kernel<D, true, NW, false>), grid, dim3(NW * 64), 0, st, a);
    else hipLaunchKernelGGL((attn_bwd_dq_kernel<D, false, NW, false>), grid, dim3(NW * 64), 0, st, a);
  }
}

template <int D>
static hipError_t bwd_d(const AttnArgs& a, bool causal, hipStream_t st) {
  // dQ first: it computes delta = rowsum(dO * O) for its query rows (one pass over O that the
  // old separate delta kernel made) and stores it for the dK/dV kernel
  if constexpr (D == 64) {
    if (dq_waves(a, D) == 8) dq_launch<D, 8>(a, causal, st);
    else dq_launch<D, 4>(a, causal, st);
  } else {
    dq_launch<D, 4>(a, causal, st);
  }
  dim3 gkv((unsigned)(((a.S + 127) / 128) * a.B * a.Hkv));
  if (bwd_ilv(D)) {
    if (causal) hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, true, true>), gkv, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, false, true>), gkv, dim3(256), 0, st, a);
  } else {
    if (causal) hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, true, false>), gkv, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, false, false>), gkv, dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t dta_attn_fwd(const AttnArgs* a, int D, bool causal, hipStream_t st) {
  if (D == 64) return fwd_d<64>(*a, causal, st);
  if (D == 128) return fwd_d<128>(*a, causal, st);
  return hipErrorInvalidValue;
}

hipError_t dta_attn_bwd(const AttnArgs* a, int D, bool causal, hipStream_t st) {
  if (D == 64) return bwd_d<64>(*a, causal, st);
  if (D == 128) return bwd_d<128>(*a, causal, st);
  return hipErrorInvalidValue;
}
