// Persistent single-workgroup train loop for the 2-layer MLP (the headline
// benchmark model, BASELINE.json: Linear(in, H) -> act -> Linear(H, out),
// SGD, 32 samples per step).
//
// Why this shape of kernel: one step of this model is ~2 MFLOP on ~45 KB of
// parameters -- three orders of magnitude below what a launch, an HBM round
// trip or a grid-wide barrier costs.  So the whole training loop runs inside
// ONE workgroup of 8 waves on one CU: the fp32 master parameters (and SGD
// momentum) are loaded into LDS once, `nsteps` full steps run back to back
// with only two workgroup barriers each, and the parameters are written back
// at the end.  Nothing is skipped: every step gathers its batch in
// DistributedSampler order, runs forward, loss, backward and the SGD update.
//
// Per step (wave w owns hidden tiles w, w+8, ...; 32 hidden units each):
//   forward  : H^T = W1 . X^T on v_mfma_f32_32x32x16_bf16 (hidden on the
//              accumulator rows, samples on the lanes; b1 is the initial
//              accumulator), act in registers, y partial = W2 . act(H) per lane
//              -> LDS                                              [barrier 1]
//   loss     : wave 0 sums the 8 partials + b2, loss (MSE / soft-target CE),
//              dY -> LDS (fp32, and bf16 into the spare columns of the batch
//              tile), b2 update; the next batch tile is written  [barrier 2]
//   backward : dH = act'(H) * (W2^T dY) lane-locally; one B operand
//              [X | 1 | dY] (32 columns) serves both weight gradients:
//                 act(H)^T . [X|1|dY] -> columns in+1.. = dW2
//                 dH^T     . [X|1|dY] -> columns 0..in-1 = dW1, column in = db1
//              (A = act(H)^T / dH^T from a wave-private LDS image through
//              ds_read_b64_tr_b16, B = the batch tile likewise), and each lane
//              applies SGD to the parameters its accumulator column owns.
// The batch of step s+1 is gathered while step s computes (index ring rows
// two steps ahead, feature rows one step ahead, both in registers).
#include "common.h"
#include "mlp_fused.h"

namespace dta {

constexpr int kMpWaves = 8;
constexpr int kMpThreads = kMpWaves * 64;
constexpr int kMpXs = 32;            // batch tile columns (bf16): X | 1 | dY | 0
constexpr int kMpImgPad = 32;
constexpr int kP2PRanks = 8;         // most ranks of an in-kernel exchange (one node)        // bf16 pad per activation-image row (rows 64 B apart mod 256 B)


__device__ __forceinline__ bf16x4 mp_tr4(const bf16* p) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

// Batch tile [32 samples][kMpXs] bf16 (64-B rows): element (row, col), its
// 16-byte chunk XOR-swizzled by (row >> 2) & 3 -- the forward's row reads
// (ds_read_b128) become conflict-free (4-way unswizzled) and the backward's
// transposed reads stay conflict-free.
__device__ __forceinline__ int xs_off(int row, int col) {
  return row * kMpXs + ((((col >> 3) ^ ((row >> 2) & 3))) << 3) + (col & 7);
}

// Natural-k-order transposed fragment of the batch tile X: lane l gets
// X[16s + 8(l>>5) + j][c0 + (l & 31)], j = 0..7.
__device__ __forceinline__ bf16x8 mp_trfrag(const bf16* X, int s, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = 16 * s + 8 * (g >> 1) + (i >> 2);
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const bf16x4 lo = mp_tr4(X + xs_off(row, col));
  const bf16x4 hi = mp_tr4(X + xs_off(row + 4, col));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// Workgroup barrier for LDS traffic only: waits for this wave's LDS ops, not
// its global loads / stores.  __syncthreads() is a release fence + s_barrier,
// and the fence waits vmcnt(0) -- it would expose the latency of the next
// batch's prefetch loads and of the per-step loss store at every barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// launch-timeline stamps (diagnostic build of one launch: dbg_step < 0), s_memrealtime (100 MHz)
#define MP_TSTAMP(k)                                                                        \
  do {                                                                                      \
    if (a.dbg && a.dbg_step < 0 && tid == 0) {                                              \
      a.dbg[64 + (k)] = __builtin_amdgcn_s_memrealtime();                                   \
      if (a.dbg_step == -2) a.dbg[72 + (k)] = __builtin_amdgcn_s_memtime();                 \
    }                                                                                       \
  } while (0)


// Activation image [32 samples][IMG]: 8-byte granules XOR-swizzled by row so
// the per-lane column writes (32 lanes = 32 rows of one granule column) spread
// over the banks instead of landing 16-way on two of them; the transposed
// reads use the same map (each lane supplies its own address).
__device__ __forceinline__ int img_off(int row, int col, int IMG) {
  return row * IMG + (((col >> 2) ^ ((row >> 1) & 7)) << 2) + (col & 3);
}

// bf16 W1 image [32 k][WS] (k >= in zero, WS = H rounded up to 64): input
// features as rows, so the forward reads its A operand (lane: hidden row h, 8
// consecutive k) with transposed reads like the gradient GEMMs', and the lane
// that owns W1[h][k] (column k of the weight-gradient accumulator, 4 consecutive
// h per register group) writes its updated rows as one 8-byte store per group
// instead of four 2-byte ones.  The 8-byte granule of (k, h) is XOR-swizzled
// within its 16-granule group by (5k) & 15 (4k ^ k): both the owners' stores and
// the transposed reads are at most 2-way (scripts/lds_banks.py model), with no
// padding, so the image costs what the old [H][32] one did.
__device__ __forceinline__ int wb_stride(int H) { return (H + 63) & ~63; }
__device__ __forceinline__ int wb_off(int h, int k, int WS) {
  return k * WS + (((h >> 2) ^ (((4 * k) ^ k) & 15)) << 2) + (h & 3);
}

__device__ __forceinline__ bf16x8 wb_trfrag(const bf16* W, int WS, int s, int h0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int k = 16 * s + 8 * (g >> 1) + (i >> 2);
  const int h = h0 + 16 * (g & 1) + 4 * (i & 3);
  const bf16x4 lo = mp_tr4(W + wb_off(h, k, WS));
  const bf16x4 hi = mp_tr4(W + wb_off(h, k + 4, WS));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ bf16x8 img_trfrag(const bf16* X, int IMG, int s, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = 16 * s + 8 * (g >> 1) + (i >> 2);
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const bf16x4 lo = mp_tr4(X + img_off(row, col, IMG));
  const bf16x4 hi = mp_tr4(X + img_off(row + 4, col, IMG));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

struct SgdH {
  float lr, mom, damp, wd;
  int nesterov, maximize, first;
};

__device__ __forceinline__ void sgd_apply(float* p, float* m, float g, const SgdH& h) {
  if (h.maximize) g = -g;
  float w = *p;
  if (h.wd != 0.f) g += h.wd * w;
  if (h.mom != 0.f) {
    const float b = h.first ? g : h.mom * (*m) + (1.f - h.damp) * g;
    *m = b;
    g = h.nesterov ? g + h.mom * b : b;
  }
  *p = w - h.lr * g;
}

// ---- DDP across ranks: one-shot gradient exchange through LL slots ----
// Every element travels as one 8-byte store {f32 bits, epoch} into slot
// [epoch & 1][rank] of EVERY rank (itself included); each rank then sums the
// `world` slots in rank order -- identical bits everywhere -- and applies SGD.
// A slot is rewritten two epochs later only after its reader consumed it (each
// element is pushed and read by the same lane mapping on every rank).
__device__ __forceinline__ void xpush(const MlpPArgs& a, unsigned ep, int off, float g) {
  const unsigned long long v = (unsigned long long)__float_as_uint(g) | ((unsigned long long)ep << 32);
  const long long slot = ((long long)(ep & 1) * a.world + a.rank) * a.slot_elems + off;
  for (int q = 0; q < a.world; ++q)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.peer_ll[q]) + slot, v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- reduce-scatter + all-gather form (xmode 2) ----
// Pushing every gradient to every rank costs world stores per element from the
// ONE workgroup that runs the loop -- at 8 ranks that single CU's store issue,
// not the xGMI links, bounds the step.  In this form each gradient goes once,
// to its owner rank (dense index j % world), into RS slot [par][src][j]; the
// owner sums its elements in rank order (the same bits as the one-shot form)
// and pushes the sum to every rank's AG slot [par][j]: 2 stores per element
// per rank instead of `world`, for one more one-way hop of latency.  Slot
// reuse is safe two epochs later for the same reason as the one-shot form.
__device__ __forceinline__ unsigned long long ll_pack(float g, unsigned ep) {
  return (unsigned long long)__float_as_uint(g) | ((unsigned long long)ep << 32);
}

__device__ __forceinline__ void xpush_owner(const MlpPArgs& a, unsigned ep, int j, float g) {
  const long long slot = ((long long)(ep & 1) * a.world + a.rank) * a.slot_elems + j;
  __hip_atomic_store(a.peer_ll[j % a.world] + slot, ll_pack(g, ep), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// bounded poll of one LL slot for tag `ep` (sticky error: see xreduce_sgd)
__device__ __forceinline__ float ll_wait(const MlpPArgs& a, const unsigned long long* p, unsigned ep) {
  unsigned long long v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  int it = 0;
  while ((unsigned)(v >> 32) != ep) {
    if (++it > a.timeout_iters ||
        ((it & 1023) == 1 && __hip_atomic_load(a.xerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      atomicOr(a.xerr, 1);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return __uint_as_float((unsigned)(v & 0xffffffffu));
}

// Sum one batch of U elements over the `W` ranks' LL slots (rank order, the
// same bits on every rank).  Every load of the batch -- R x U uncached
// system-scope reads -- is issued before any tag is checked, so a batch costs
// one memory latency instead of one per rank; a slot whose tag is not yet `ep`
// is re-polled.  Unused (rank, element) pairs load a valid duplicate address
// (no branch around a load) and are left out of the sum.
template <int R, int U>
__device__ __forceinline__ void ll_sum_ranks(const MlpPArgs& a, const unsigned long long* base, long long stride,
                                             const long long (&idx)[U], const bool (&live)[U], int W, unsigned ep,
                                             float (&acc)[U]) {
  unsigned long long v[R][U];
#pragma unroll
  for (int q = 0; q < R; ++q)
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[q][u] = __hip_atomic_load(base + (long long)(q < W ? q : 0) * stride + idx[u], __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = 0.f;
#pragma unroll
  for (int q = 0; q < R; ++q)
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (q < W && live[u]) {
        float x = __uint_as_float((unsigned)(v[q][u] & 0xffffffffu));
        if ((unsigned)(v[q][u] >> 32) != ep) x = ll_wait(a, base + (long long)q * stride + idx[u], ep);
        acc[u] += x;
      }
}

// owner: sum the elements j = rank, rank + world, ... over the RS slots (rank
// order) and push each sum to every rank's AG slot
__device__ void xowner_reduce(const MlpPArgs& a, unsigned ep, int n) {
  constexpr int U = 4;
  const int W = a.world, par = ep & 1;
  const unsigned long long* rs = a.local_ll + (long long)par * W * a.slot_elems;
  const long long ag = 2LL * W * a.slot_elems + (long long)par * a.slot_elems;
  const int nown = (n - a.rank + W - 1) / W;
  for (int k0 = threadIdx.x; k0 < nown; k0 += kMpThreads * U) {
    float acc[U];
    long long idx[U];
    bool live[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * kMpThreads;
      live[u] = k < nown;
      idx[u] = a.rank + (long long)(live[u] ? k : 0) * W;
    }
    ll_sum_ranks<kP2PRanks, U>(a, rs, a.slot_elems, idx, live, W, ep, acc);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * kMpThreads;
      if (k < nown) {
        const unsigned long long v = ll_pack(acc[u], ep);
        for (int q = 0; q < W; ++q)
          __hip_atomic_store(a.peer_ll[q] + ag + a.rank + (long long)k * W, v, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// flat offset of the j-th real parameter (W1 | b1 | W2 | b2, padding skipped)
__device__ __forceinline__ int xoff(const MlpPArgs& a, int j) {
  const int n1 = a.hidden * a.in_dim;
  if (j < n1) return a.o_w1 + j;
  j -= n1;
  if (j < a.hidden) return a.o_b1 + j;
  j -= a.hidden;
  if (j < a.hidden) return a.o_w2 + j;
  return a.o_b2 + (j - a.hidden);
}

// AG: read the summed gradient of dense element j from this rank's AG slot
// (xmode 2); otherwise sum the one-shot slots [par][q][offset] in rank order.
template <bool PLAIN, bool AG>
__device__ void xreduce_sgd(const MlpPArgs& a, unsigned ep, float* Pf, float* Mf, bf16* Wb, SgdH hs, int first) {
  constexpr int U = AG ? 8 : 4;  // elements per thread per batch (x ranks loads in flight)
  hs.first = first;
  const int n = a.hidden * a.in_dim + 2 * a.hidden + a.out_dim;
  const int W = AG ? 1 : a.world, par = ep & 1;
  const unsigned long long* base = AG ? a.local_ll + 2LL * a.world * a.slot_elems + (long long)par * a.slot_elems
                                      : a.local_ll + (long long)par * W * a.slot_elems;
  for (int j0 = threadIdx.x; j0 < n; j0 += kMpThreads * U) {
    int off[U];
    float acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * kMpThreads;
      off[u] = xoff(a, j < n ? j : n - 1);
      acc[u] = 0.f;
    }
    {
      long long idx[U];
      bool live[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + u * kMpThreads;
        live[u] = true;  // j >= n duplicates element n-1 and is not applied below
        idx[u] = AG ? (long long)(j < n ? j : n - 1) : (long long)off[u];
      }
      ll_sum_ranks<AG ? 1 : kP2PRanks, U>(a, base, a.slot_elems, idx, live, W, ep, acc);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * kMpThreads;
      if (j < n) {
        const int o = off[u];
        float g = acc[u];
        float p = Pf[o];
        if (!PLAIN) {
          if (hs.maximize) g = -g;
          if (hs.wd != 0.f) g += hs.wd * p;
          if (hs.mom != 0.f) {
            const float b = hs.first ? g : hs.mom * Mf[o] + (1.f - hs.damp) * g;
            Mf[o] = b;
            g = hs.nesterov ? g + hs.mom * b : b;
          }
        }
        p -= hs.lr * g;
        Pf[o] = p;
        if (j < a.hidden * a.in_dim) Wb[wb_off(j / a.in_dim, j % a.in_dim, wb_stride(a.hidden))] = f2bf(p);
      }
    }
  }
}

// ---- helper-workgroup exchange (xmode 3) ----
// The loop's single CU issues every global access of the exchange itself in
// the other forms, and one CU's load/store rate (not xGMI) then sets the step
// time.  Here the loop writes its gradients ONCE (fp32, fragment order: tile,
// accumulator register, lane -- 256 contiguous bytes per wave-instruction)
// and releases them with a flag; nh helper workgroups on other CUs each take a
// slice, push it to every rank's LL slots, sum the world slices in rank order
// and hand the sums back through xg_red + a per-helper flag.  Gradient bytes
// through the loop's CU per step: 2 x 64 KB, whatever the world size.
// Visibility: every access to the hand-off bytes and flags is a system-scope
// (sc1) load / store -- the per-XCD L2s are not coherent with each other, and
// the loop and a helper may sit on different XCDs -- in the p2p buffer's
// uncached regions: writer waves drain vmcnt, barrier, then the flag store;
// the reader issues its loads only after the poll returned.  No L2 write-back
// or invalidate per step (an acquire in the poll loop would invalidate L2 on
// every iteration).  One poller per flag matters: an LL hand-off (every thread
// polling its own {value, epoch} slot, no flags) measured 1.5-1.7x slower --
// thousands of threads spinning on uncached slots load the memory system.
__device__ __forceinline__ float ld_sc(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sc(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool flag_wait(const MlpPArgs& a, const int* f, int ep) {
  int it = 0;
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != ep) {
    if (++it > a.timeout_iters ||
        ((it & 1023) == 1 && __hip_atomic_load(a.xerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      atomicOr(a.xerr, 1);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

__device__ void helper_loop(const MlpPArgs& a, unsigned xe0) {
  // helper h owns elements [512 h, 512 h + 512): half of tile h / 2, written by
  // loop wave (h / 2) % 8 -- or the output-bias gradients (last helper, wave 0)
  const int h = blockIdx.x - 1, tid = threadIdx.x;
  const int e0 = h * kMpThreads, e1 = min(a.xe, e0 + kMpThreads);
  const int NT = a.hidden / 32;
  const int owner = h < 2 * NT ? (h >> 1) % kMpWaves : 0;
  const int W = a.world;
  constexpr int U = 1;  // one element per thread
  for (int s = 0; s < a.nsteps; ++s) {
    const unsigned ep = xe0 + s + 1;
    const int par = ep & 1;
    if (tid == 0) flag_wait(a, a.xready + par * kMpWaves + owner, (int)ep);
    __syncthreads();
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + tid + u * kMpThreads;
      v[u] = e < e1 ? ld_sc(a.xg_out + (long long)par * a.xe + e) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + tid + u * kMpThreads;
      if (e < e1) {
        const unsigned long long pv = ll_pack(v[u], ep);
        const long long slot = ((long long)par * W + a.rank) * a.slot_elems + e;
        for (int q = 0; q < W; ++q)
          __hip_atomic_store(a.peer_ll[q] + slot, pv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    float acc[U];
    long long idx[U];
    bool live[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + tid + u * kMpThreads;
      live[u] = e < e1;
      idx[u] = live[u] ? e : e0;
    }
    const unsigned long long* base = a.local_ll + (long long)par * W * a.slot_elems;
    ll_sum_ranks<kP2PRanks, U>(a, base, a.slot_elems, idx, live, W, ep, acc);  // rank order
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + tid + u * kMpThreads;
      if (e < e1) st_sc(a.xg_red + (long long)par * a.xe + e, acc[u]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(a.xdone + h, (int)ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// OUT: output width, TPW: hidden tiles per wave (H <= 256 TPW), PLAIN: SGD
// without momentum / weight decay / maximize (the update is p -= lr * g)
// XM: 0 one rank, else the exchange form (1 one-shot, 2 rs+ag, 3 helpers) -- one
// instantiation per form keeps the other forms' live ranges out of its registers
template <int ACT, int OUT, int TPW, bool PLAIN, int XM>
__global__ void __launch_bounds__(kMpThreads) mlp_persistent_kernel(MlpPArgs a) {
  static_assert(OUT == 1, "the persistent loop serves single-output heads");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int IN = a.in_dim, H = a.hidden, B = a.B, NT = H / 32;
  const int IMG = H + kMpImgPad;  // activation image row stride (elements)
  if (XM == 3 && blockIdx.x > 0) {  // xmode 3: helper workgroups (the loop is workgroup 0)
    helper_loop(a, (unsigned)*a.xepoch);
    return;
  }

  constexpr bool multi = XM != 0;  // DDP across ranks (a.world > 1)
  // ---- LDS carve ----
  float* Pf = reinterpret_cast<float*>(smem);                       // [total]
  float* Mf = Pf + a.total;  // [total] momenta, several ranks only (one rank: registers)
  char* q = reinterpret_cast<char*>(Mf + (a.M && multi ? a.total : 0));
  bf16* Xs = reinterpret_cast<bf16*>(q);                            // [2][32][kMpXs]
  q += 2 * 32 * kMpXs * 2;
  bf16* Img = reinterpret_cast<bf16*>(q);                           // [32][IMG]
  q += 32 * IMG * 2;
  float* Ypart = reinterpret_cast<float*>(q);                       // [waves][OUT][32]
  q += kMpWaves * OUT * 32 * 4;
  float* dYf = reinterpret_cast<float*>(q);                         // [OUT][32]
  q += OUT * 32 * 4;
  float* Ts = reinterpret_cast<float*>(q);                          // [2][32][OUT]
  q += 2 * 32 * OUT * 4;
  float* lossbuf = reinterpret_cast<float*>(q);                     // [1]
  q += 16;
  bf16* Wb = reinterpret_cast<bf16*>(q);                            // [32][WS] bf16 W1^T (k >= in zero)
  const int WS = wb_stride(H);

  int c0 = *a.cursor;
  int lcur = *a.loss_cursor;
  int first = a.M ? (*a.mom_started == 0) : 0;
  const unsigned xe0 = multi ? (unsigned)*a.xepoch : 0u;

  // ---- batch pipeline: idx two steps ahead, features one step ahead ----
  // threads [256, 256 + 32): idx of sample r for a step; feature loads: sample = tid-256 (r < B)
  const bool gthr = tid >= 256 && tid < 256 + 32;
  const int gr = tid - 256;
  auto ring_row = [&](int s) { return (c0 + s) % a.ring_steps; };
  int idx_next = 0;     // sample index of row gr for step s+1
  bf16x8 xv[4];         // padded feature row gr of step s+1 (X | 1 | 0), 4 x 16-B loads, no branches
  float tv[OUT];
  const bf16* Xp = static_cast<const bf16*>(a.Xp);
  // unconditional loads (a select around a load makes hipcc wait vmcnt(0) on it):
  // ring rows are always allocated; samples >= B re-read column B-1 and are masked at the store
  const int gcol = gr < B ? gr : B - 1;
  auto load_idx = [&](int s) -> int { return a.idx_ring[(int64_t)ring_row(s) * a.idx_stride + gcol]; };
  auto load_rows = [&](int sample) {
    const bf16x8* xr = reinterpret_cast<const bf16x8*>(Xp + (int64_t)sample * kMpXs);
#pragma unroll
    for (int c = 0; c < 4; ++c) xv[c] = xr[c];
#pragma unroll
    for (int o = 0; o < OUT; ++o) tv[o] = a.T[(int64_t)sample * OUT + o];
  };
  auto store_rows = [&](int buf) {
    // row gr of the batch tile: X | 1 | 0 (the dY columns are written by the loss phase)
    bf16* tile = Xs + buf * 32 * kMpXs;
    const bool live = gr < B;
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = f2bf(0.f);
#pragma unroll
    for (int c = 0; c < 4; ++c) *reinterpret_cast<bf16x8*>(tile + xs_off(gr, 8 * c)) = live ? xv[c] : z;
#pragma unroll
    for (int o = 0; o < OUT; ++o) Ts[(buf * 32 + gr) * OUT + o] = live ? tv[o] : 0.f;
  };
  // the first batch's dependent loads (index -> feature row) are issued before the
  // parameter loads, so their two round trips overlap the parameter fetch
  if (gthr) {
    load_rows(load_idx(0));
    idx_next = load_idx(1);
  }
  MP_TSTAMP(0);
  // ---- load parameters (+ momentum), build the bf16 W1 fragment image ----
  // All of a thread's 16-B loads are issued before any LDS store (indices clamped,
  // stores masked: no select around a load), so the ~45 KB arrive in one HBM round
  // trip instead of one dependent miss per loop iteration (that was ~20 us of fixed
  // cost per launch, a fifth of a 20-step launch).
  {
    const int nv = a.total >> 2;  // whole float4s; P / M are 16-B aligned allocations
    const float4* P4 = reinterpret_cast<const float4*>(a.P);
    const float4* M4 = reinterpret_cast<const float4*>(a.M);
    constexpr int kLd = 8;
    for (int base = 0; base < nv; base += kMpThreads * kLd) {
      float4 pv[kLd], mv[kLd];
#pragma unroll
      for (int j = 0; j < kLd; ++j) pv[j] = P4[min(base + j * kMpThreads + tid, nv - 1)];
      if (multi && a.M) {
#pragma unroll
        for (int j = 0; j < kLd; ++j) mv[j] = M4[min(base + j * kMpThreads + tid, nv - 1)];
      }
#pragma unroll
      for (int j = 0; j < kLd; ++j) {
        const int i = base + j * kMpThreads + tid;
        if (i < nv) {
          Pf[4 * i] = pv[j].x; Pf[4 * i + 1] = pv[j].y; Pf[4 * i + 2] = pv[j].z; Pf[4 * i + 3] = pv[j].w;
          if (multi && a.M) {
            Mf[4 * i] = mv[j].x; Mf[4 * i + 1] = mv[j].y; Mf[4 * i + 2] = mv[j].z; Mf[4 * i + 3] = mv[j].w;
          }
        }
      }
    }
    for (int i = 4 * nv + tid; i < a.total; i += kMpThreads) {
      Pf[i] = a.P[i];
      if (multi && a.M) Mf[i] = a.M[i];
    }
  }
  __syncthreads();
  MP_TSTAMP(1);
  for (int i = tid; i < 32 * (WS / 4); i += kMpThreads) {  // from the LDS copy: no second HBM pass
    const int k = i / (WS / 4), h = 4 * (i % (WS / 4));       // 4 consecutive h of input feature k
    if (h >= H) continue;
    bf16x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = f2bf(k < IN ? Pf[a.o_w1 + (h + j) * IN + k] : 0.f);
    *reinterpret_cast<bf16x4*>(Wb + wb_off(h, k, WS)) = v;
  }
  if (gthr) store_rows(0);
  if (tid == 0) *lossbuf = 0.f;
  __syncthreads();
  MP_TSTAMP(2);

  const SgdH hbase{a.lr, a.momentum, a.dampening, a.weight_decay, a.nesterov, a.maximize, 0};
  // One rank: the fp32 master parameters (and momenta) a lane updates stay in its
  // registers for the whole launch -- lane (column c = lane & 31) of wave w owns, for
  // each of its tiles, the 16 accumulator rows of column c of the gradient GEMMs
  // (W1[h][c], b1[h] or W2[h]); the LDS copy is only the forward's view of b1 / W2
  // and the bf16 W1 image.  Written back to LDS after the loop.
  const int own_c = r32;
  const bool own = own_c <= IN + 1;
  const int own_base = own_c < IN ? a.o_w1 + own_c : (own_c == IN ? a.o_b1 : a.o_w2);
  const int own_stride = own_c < IN ? IN : 1;
  float preg[TPW][16], mreg[TPW][16];
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      preg[tt][i] = 0.f;
      mreg[tt][i] = 0.f;
    }
  if constexpr (!multi) {
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      const int t = wave + kMpWaves * tt;
      if (t < NT && own) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int off = own_base + (t * 32 + mfma32_row(i, lane)) * own_stride;
          preg[tt][i] = Pf[off];
          if (!PLAIN && a.M) mreg[tt][i] = a.M[off];
        }
      }
    }
  }
  const float lscale = (a.loss_type == LOSS_MSE) ? 1.f / (float)(B * OUT) : 1.f / (float)B;

  float dy_keep[OUT], loss_keep = 0.f;  // one rank: wave 0's dY / loss, finished after its backward
  float mb2[OUT];                       // one rank: the output bias' momenta (wave 0, lane 0)
#pragma unroll
  for (int o = 0; o < OUT; ++o) mb2[o] = (!multi && !PLAIN && a.M && tid == 0) ? a.M[a.o_b2 + o] : 0.f;
#pragma unroll
  for (int o = 0; o < OUT; ++o) dy_keep[o] = 0.f;
  for (int s = 0; s < a.nsteps; ++s) {
    const int cb = s & 1;
    const bf16* Xb = Xs + cb * 32 * kMpXs;
    // prefetch: features of step s+1, index of step s+2
    if (gthr && s + 1 < a.nsteps) {
      load_rows(idx_next);
      idx_next = load_idx(s + 2);
    }
    // ================= forward (own tiles) =================
    float yp[OUT];
#pragma unroll
    for (int o = 0; o < OUT; ++o) yp[o] = 0.f;
    // B operand X^T: lane (col = sample r32), k = 16ks + 8hh + j  (row read of the batch tile)
    const bf16x8 xb0 = *reinterpret_cast<const bf16x8*>(Xb + xs_off(r32, hh * 8));
    const bf16x8 xb1 = *reinterpret_cast<const bf16x8*>(Xb + xs_off(r32, 16 + hh * 8));
    f32x16 hpre[TPW];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      const int t = wave + kMpWaves * tt;
      if (t < NT) {
        const int h0 = t * 32;
        f32x16 acc;
        // b1 as the initial accumulator: rows 8g + 4hh + 0..3 are consecutive -> float4 reads
        float w2v[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 bv = *reinterpret_cast<const float4*>(Pf + a.o_b1 + h0 + 8 * g + 4 * hh);
          const float4 wv = *reinterpret_cast<const float4*>(Pf + a.o_w2 + h0 + 8 * g + 4 * hh);
          acc[4 * g] = bv.x; acc[4 * g + 1] = bv.y; acc[4 * g + 2] = bv.z; acc[4 * g + 3] = bv.w;
          w2v[4 * g] = wv.x; w2v[4 * g + 1] = wv.y; w2v[4 * g + 2] = wv.z; w2v[4 * g + 3] = wv.w;
        }
        // A operand W1: lane (row h = h0 + r32), k = 16ks + 8hh + j: one 16-B read of the bf16 image
        acc = mfma32x32x16(wb_trfrag(Wb, WS, 0, h0, lane), xb0, acc);
        acc = mfma32x32x16(wb_trfrag(Wb, WS, 1, h0, lane), xb1, acc);
        hpre[tt] = acc;
        // layer 2 partial: y[sample] += W2[h] * act(hpre[h][sample]) over this lane's 16 rows
#pragma unroll
        for (int i = 0; i < 16; ++i) yp[0] += w2v[i] * (ACT == ACT_RELU ? relu1(acc[i]) : act_fwd(ACT, acc[i]));
      }
    }
#pragma unroll
    for (int o = 0; o < OUT; ++o) {
      yp[o] += __shfl_xor(yp[o], 32, kWave);
      if (hh == 0) Ypart[(wave * OUT + o) * 32 + r32] = yp[o];
    }
    lds_barrier();  // ---------------- barrier 1
    // ================= loss, dY, b2 (wave 0); next batch tile (staging threads) =================
    if (wave == 0) {
      const int r = r32;
      float lossr = 0.f;
      float dy[OUT];
      if (hh == 0 && r < B) {
        float y[OUT], t[OUT];
#pragma unroll
        for (int o = 0; o < OUT; ++o) {
          float acc = Pf[a.o_b2 + o];
#pragma unroll
          for (int w = 0; w < kMpWaves; ++w) acc += Ypart[(w * OUT + o) * 32 + r];
          y[o] = acc;
          t[o] = Ts[(cb * 32 + r) * OUT + o];
        }
        if (a.loss_type == LOSS_MSE) {
#pragma unroll
          for (int o = 0; o < OUT; ++o) {
            const float d = y[o] - t[o];
            lossr += d * d;
            dy[o] = 2.f * d * lscale;
          }
        } else {
          float m = -INFINITY, sx = 0.f, tsum = 0.f;
#pragma unroll
          for (int o = 0; o < OUT; ++o) m = fmaxf(m, y[o]);
#pragma unroll
          for (int o = 0; o < OUT; ++o) {
            sx += __expf(y[o] - m);
            tsum += t[o];
          }
          const float lse = m + __logf(sx);
#pragma unroll
          for (int o = 0; o < OUT; ++o) {
            lossr -= t[o] * (y[o] - lse);
            dy[o] = (__expf(y[o] - lse) * tsum - t[o]) * lscale;
          }
        }
      } else {
#pragma unroll
        for (int o = 0; o < OUT; ++o) dy[o] = 0.f;
      }
      // grads are averaged over ranks by the caller's grad_scale (1 for one rank)
#pragma unroll
      for (int o = 0; o < OUT; ++o) dy[o] *= a.grad_scale;
      if (hh == 0) {
#pragma unroll
        for (int o = 0; o < OUT; ++o) {
          dYf[o * 32 + r] = dy[o];
          const_cast<bf16*>(Xb)[xs_off(r, IN + 1 + o)] = f2bf(dy[o]);
        }
      }
      if constexpr (multi) {
        // db2 = sum over samples, pushed into the exchange with the other gradients; loss
#pragma unroll
        for (int o = 0; o < OUT; ++o) {
          const float db = wave_sum(hh == 0 ? dy[o] : 0.f);
          if (lane == 0) {
            if (XM == 3) st_sc(a.xg_out + (long long)((xe0 + s + 1) & 1) * a.xe + NT * 1024 + o, db);
            else if (XM == 2) xpush_owner(a, xe0 + s + 1, a.hidden * IN + 2 * a.hidden + o, db);
            else xpush(a, xe0 + s + 1, a.o_b2 + o, db);
          }
        }
        const float lsum = wave_sum(hh == 0 ? lossr : 0.f);
        if (lane == 0) {
          a.loss_ring[lcur % a.loss_len] = lsum * lscale;
          ++lcur;
        }
      } else {
        // one rank: only wave 0 reads b2, so its update (and the loss sum) wait
        // for the tail of wave 0's backward instead of holding every wave at barrier 2
#pragma unroll
        for (int o = 0; o < OUT; ++o) dy_keep[o] = hh == 0 ? dy[o] : 0.f;
        loss_keep = hh == 0 ? lossr : 0.f;
      }
    }
    if (gthr && s + 1 < a.nsteps) store_rows(cb ^ 1);
    lds_barrier();  // ---------------- barrier 2
    // ================= backward + SGD (own tiles) =================
    SgdH hs = hbase;
    hs.first = first;
    const float dyv = dYf[r32];
    // parameter owned by accumulator column c = r32 at hidden row h: p[base + h * stride]
    //   c < IN: W1[h][c] (from dW1 = C1)   c == IN: b1[h] (C1)   c == IN + 1: W2[0][h] (C2)
    const int c = r32;
    const bool upd = c <= IN + 1;
    const int pbase = c < IN ? a.o_w1 + c : (c == IN ? a.o_b1 : a.o_w2);
    const int pstride = c < IN ? IN : 1;
    // B operand [X | 1 | dY] of both gradient GEMMs (same for every tile)
    const bf16x8 xf0 = mp_trfrag(Xb, 0, 0, lane), xf1 = mp_trfrag(Xb, 1, 0, lane);
    // ONE accumulator per tile for both weight gradients: act(H)^T . [0 | 0 | dY] then
    // dH^T . [X | 1 | 0] -- column c of the sum is dW2 for c == in + 1 and dW1 / db1 for
    // c <= in, so every owner lane reads its gradient from the same registers (no
    // per-element select between two accumulators)
    const bool dycol = c == IN + 1;
    bf16x8 yf0, yf1, zf0, zf1;  // (one rank; the exchange forms select between two accumulators)
#pragma unroll
    for (int j = 0; j < 8 && !multi; ++j) {
      yf0[j] = dycol ? xf0[j] : f2bf(0.f);
      yf1[j] = dycol ? xf1[j] : f2bf(0.f);
      zf0[j] = dycol ? f2bf(0.f) : xf0[j];
      zf1[j] = dycol ? f2bf(0.f) : xf1[j];
    }
    // One rank: ONE accumulator per tile for both weight gradients (masked B operands
    // above); the exchange forms select between two (their push code needs the
    // registers the masked operands take).
    if constexpr (!multi) {
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      const int t = wave + kMpWaves * tt;
      if (t < NT) {
        const int h0 = t * 32;
        f32x16 dh;
        // act(H) -> image columns [h0, h0+32): lane (sample r32) writes rows 8g+4hh..+3 of its column
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 wv = *reinterpret_cast<const float4*>(Pf + a.o_w2 + h0 + 8 * g + 4 * hh);  // pre-update W2
          const float w2g[4] = {wv.x, wv.y, wv.z, wv.w};
          float av[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int i = 4 * g + e;
            const float x = hpre[tt][i];
            if constexpr (ACT == ACT_RELU) {  // max, mul, compare + mask (a select here became a branch
              av[e] = relu1(x);                // around the W2 load)
              const float prod = w2g[e] * dyv;
              dh[i] = __builtin_bit_cast(float, __builtin_bit_cast(int, prod) & (x > 0.f ? -1 : 0));
            } else {
              av[e] = act_fwd(ACT, x);
              dh[i] = w2g[e] * dyv * act_bwd(ACT, x);
            }
          }
          *reinterpret_cast<bf16x4*>(Img + img_off(r32, h0 + 8 * g + 4 * hh, IMG)) = pk4_bf16(av[0], av[1], av[2], av[3]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        f32x16 gacc;  // act(H)^T . [0 | 0 | dY], then += dH^T . [X | 1 | 0]
#pragma unroll
        for (int i = 0; i < 16; ++i) gacc[i] = 0.f;
        gacc = mfma32x32x16(img_trfrag(Img, IMG, 0, h0, lane), yf0, gacc);
        gacc = mfma32x32x16(img_trfrag(Img, IMG, 1, h0, lane), yf1, gacc);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // act(H) reads done before dH overwrites the image
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<bf16x4*>(Img + img_off(r32, h0 + 8 * g + 4 * hh, IMG)) =
              pk4_bf16(dh[4 * g], dh[4 * g + 1], dh[4 * g + 2], dh[4 * g + 3]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        gacc = mfma32x32x16(img_trfrag(Img, IMG, 0, h0, lane), zf0, gacc);
        gacc = mfma32x32x16(img_trfrag(Img, IMG, 1, h0, lane), zf1, gacc);
        if (upd) {
          // one rank: register-resident parameters (see the prologue); only b1 / W2 go
          // back to LDS (the forward's and the next backward's view), W1 to its bf16 image
          const bool w1col = c < IN;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float g = gacc[i];
            if (!PLAIN) {
              if (hs.maximize) g = -g;
              if (hs.wd != 0.f) g += hs.wd * preg[tt][i];
              if (hs.mom != 0.f) {
                mreg[tt][i] = hs.first ? g : hs.mom * mreg[tt][i] + (1.f - hs.damp) * g;
                g = hs.nesterov ? g + hs.mom * mreg[tt][i] : mreg[tt][i];
              }
            }
            preg[tt][i] -= hs.lr * g;
          }
          if (w1col) {
#pragma unroll
            for (int g = 0; g < 4; ++g)  // rows h0 + 8g + 4hh + 0..3
              *reinterpret_cast<bf16x4*>(Wb + wb_off(h0 + 8 * g + 4 * hh, c, WS)) =
                  pk4_bf16(preg[tt][4 * g], preg[tt][4 * g + 1], preg[tt][4 * g + 2], preg[tt][4 * g + 3]);
          } else {
            // rows 8g + 4hh + 0..3 are consecutive: 16-byte stores
            float* dst = Pf + pbase + h0 + 4 * hh;
#pragma unroll
            for (int g = 0; g < 4; ++g)
              *reinterpret_cast<float4*>(dst + 8 * g) =
                  make_float4(preg[tt][4 * g], preg[tt][4 * g + 1], preg[tt][4 * g + 2], preg[tt][4 * g + 3]);
          }
        }
      }
    }
    } else {
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      const int t = wave + kMpWaves * tt;
      if (t < NT) {
        const int h0 = t * 32;
        f32x16 dh;
        // act(H) -> image columns [h0, h0+32): lane (sample r32) writes rows 8g+4hh..+3 of its column
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 wv = *reinterpret_cast<const float4*>(Pf + a.o_w2 + h0 + 8 * g + 4 * hh);  // pre-update W2
          const float w2g[4] = {wv.x, wv.y, wv.z, wv.w};
          float av[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int i = 4 * g + e;
            const float x = hpre[tt][i];
            if constexpr (ACT == ACT_RELU) {
              av[e] = relu1(x);
              const float prod = w2g[e] * dyv;
              dh[i] = __builtin_bit_cast(float, __builtin_bit_cast(int, prod) & (x > 0.f ? -1 : 0));
            } else {
              av[e] = act_fwd(ACT, x);
              dh[i] = w2g[e] * dyv * act_bwd(ACT, x);
            }
          }
          *reinterpret_cast<bf16x4*>(Img + img_off(r32, h0 + 8 * g + 4 * hh, IMG)) = pk4_bf16(av[0], av[1], av[2], av[3]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // gradient GEMMs: rows = hidden units of this tile, columns = [X | 1 | dY]
        f32x16 c2, c1;
#pragma unroll
        for (int i = 0; i < 16; ++i) c2[i] = c1[i] = 0.f;
        c2 = mfma32x32x16(img_trfrag(Img, IMG, 0, h0, lane), xf0, c2);
        c2 = mfma32x32x16(img_trfrag(Img, IMG, 1, h0, lane), xf1, c2);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // act(H) reads done before dH overwrites the image
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<bf16x4*>(Img + img_off(r32, h0 + 8 * g + 4 * hh, IMG)) =
              pk4_bf16(dh[4 * g], dh[4 * g + 1], dh[4 * g + 2], dh[4 * g + 3]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        c1 = mfma32x32x16(img_trfrag(Img, IMG, 0, h0, lane), xf0, c1);
        c1 = mfma32x32x16(img_trfrag(Img, IMG, 1, h0, lane), xf1, c1);
        if (multi && (upd || XM == 3)) {
          // DDP: this rank's (1/world-scaled) gradient to every rank's slot [par][rank]
          const unsigned ep = xe0 + s + 1;
          if (XM == 3) {
            // fragment order: [tile][register][lane]; lanes past the parameter columns write 0
            float* go = a.xg_out + (long long)(ep & 1) * a.xe + (long long)t * 1024 + lane;
#pragma unroll
            for (int i = 0; i < 16; ++i) st_sc(go + i * 64, upd ? ((dycol ? c2[i] : c1[i])) : 0.f);
          } else if (XM == 2) {
            // dense index: W1[h][c] = h * IN + c, b1[h] = H IN + h, W2[h] = H IN + H + h
            const int jb = c < IN ? c : H * IN + (c - IN) * H;
            const int js = c < IN ? IN : 1;
#pragma unroll
            for (int i = 0; i < 16; ++i)
              xpush_owner(a, ep, jb + (h0 + mfma32_row(i, lane)) * js, (dycol ? c2[i] : c1[i]));
          } else {
#pragma unroll
            for (int i = 0; i < 16; ++i)
              xpush(a, ep, pbase + (h0 + mfma32_row(i, lane)) * pstride, (dycol ? c2[i] : c1[i]));
          }
        }
      }
    }
    }
    if constexpr (XM != 0) {
      // all waves done reading the pre-update parameters before any update
      if (XM == 3) {
        // per-wave hand-off, no workgroup barrier: a wave's tiles (and wave 0's
        // output-bias gradient) go to their own helpers and come back from them,
        // and the wave updates only parameters it alone reads next step (as on
        // one rank), so fast waves run ahead
        const unsigned ep = xe0 + s + 1;
        const int par = ep & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's gradient stores landed
        if (lane == 0)
          __hip_atomic_store(a.xready + par * kMpWaves + wave, (int)ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (lane < 2 * TPW) {
          const int t = wave + kMpWaves * (lane >> 1);
          if (t < NT) flag_wait(a, a.xdone + 2 * t + (lane & 1), (int)ep);
        } else if (lane == 2 * TPW && wave == 0) {
          flag_wait(a, a.xdone + 2 * NT, (int)ep);
        }
        // SGD from the summed gradients (same lane <-> parameter map as one rank)
        const float* gr = a.xg_red + (long long)par * a.xe;
        SgdH hs2 = hbase;
        hs2.first = first;
        // all of this lane's summed gradients in flight at once (one latency)
        float gall[TPW][16];
#pragma unroll
        for (int tt = 0; tt < TPW; ++tt) {
          const int t = wave + kMpWaves * tt;
#pragma unroll
          for (int i = 0; i < 16; ++i) gall[tt][i] = t < NT ? ld_sc(gr + (long long)t * 1024 + i * 64 + lane) : 0.f;
        }
#pragma unroll
        for (int tt = 0; tt < TPW; ++tt) {
          const int t = wave + kMpWaves * tt;
          if (t < NT && upd) {
            const int h0 = t * 32;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
              float pv[8], mv[8], gv[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int i = 8 * half + u;
                const int off = pbase + (h0 + mfma32_row(i, lane)) * pstride;
                gv[u] = gall[tt][i];
                pv[u] = Pf[off];
                mv[u] = PLAIN ? 0.f : Mf[off];
              }
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                float g = gv[u];
                if (!PLAIN) {
                  if (hs2.maximize) g = -g;
                  if (hs2.wd != 0.f) g += hs2.wd * pv[u];
                  if (hs2.mom != 0.f) {
                    mv[u] = hs2.first ? g : hs2.mom * mv[u] + (1.f - hs2.damp) * g;
                    g = hs2.nesterov ? g + hs2.mom * mv[u] : mv[u];
                  }
                }
                pv[u] -= hs2.lr * g;
              }
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int hrow = h0 + mfma32_row(8 * half + u, lane);
                const int off = pbase + hrow * pstride;
                Pf[off] = pv[u];
                if (!PLAIN && hs2.mom != 0.f) Mf[off] = mv[u];
                if (c < IN) Wb[wb_off(hrow, c, WS)] = f2bf(pv[u]);
              }
            }
          }
        }
        if (tid < a.out_dim) sgd_apply(Pf + a.o_b2 + tid, Mf + a.o_b2 + tid, ld_sc(gr + NT * 1024 + tid), hs2);
      } else if (XM == 2) {
        // the owner sums need no LDS: start them before the barrier
        xowner_reduce(a, xe0 + s + 1, H * IN + 2 * H + a.out_dim);
        lds_barrier();
        xreduce_sgd<PLAIN, true>(a, xe0 + s + 1, Pf, Mf, Wb, hbase, first);
      } else {
        lds_barrier();
        xreduce_sgd<PLAIN, false>(a, xe0 + s + 1, Pf, Mf, Wb, hbase, first);
      }
      if (XM != 3) lds_barrier();
    }
    if constexpr (!multi) {
      if (wave == 0) {  // the deferred output-bias update and loss of this step (see the loss phase)
#pragma unroll
        for (int o = 0; o < OUT; ++o) {
          const float db = wave_sum(dy_keep[o]);
          if (lane == 0) {
            SgdH hb = hbase;
            hb.first = first;
            sgd_apply(Pf + a.o_b2 + o, &mb2[o], db, hb);
          }
        }
        const float lsum = wave_sum(loss_keep);
        if (lane == 0) {
          a.loss_ring[lcur % a.loss_len] = lsum * lscale;
          ++lcur;
        }
      }
    }
    first = 0;
    // one rank: no barrier here -- the next forward reads only this wave's own
    // rows of W1 / b1 / W2 (updated above by this wave) and b2 / the next batch
    // tile, both published before barrier 2 of this step
  }
  if constexpr (!multi) {  // register-resident parameters back into the LDS copy
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      const int t = wave + kMpWaves * tt;
      if (t < NT && own) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int off = own_base + (t * 32 + mfma32_row(i, lane)) * own_stride;
          Pf[off] = preg[tt][i];
          if (!PLAIN && a.M) a.M[off] = mreg[tt][i];
        }
      }
    }
  }
  __syncthreads();
  MP_TSTAMP(3);
  for (int i = tid; i < a.total; i += kMpThreads) {
    a.P[i] = Pf[i];
    if (multi && a.M) a.M[i] = Mf[i];
  }
  if (!multi && !PLAIN && a.M && tid == 0) {
#pragma unroll
    for (int o = 0; o < OUT; ++o) a.M[a.o_b2 + o] = mb2[o];
  }
  if (tid == 0) {
    if (multi) *a.xepoch = (int)(xe0 + (unsigned)a.nsteps);
    *a.cursor = (c0 + a.nsteps) % a.ring_steps;
    *a.loss_cursor = lcur;
    if (a.M && a.nsteps > 0) *a.mom_started = 1;
  }
  MP_TSTAMP(4);
}

}  // namespace dta

using namespace dta;

size_t dta_mlp_persistent_lds_bytes(int total, int hidden, int out_dim, int has_mom) {
  return (size_t)total * 4 * (has_mom ? 2 : 1) + 2 * 32 * kMpXs * 2 + 32 * (hidden + kMpImgPad) * 2 +
         kMpWaves * out_dim * 32 * 4 + out_dim * 32 * 4 + 2 * 32 * out_dim * 4 + 16 +
         (size_t)32 * ((hidden + 63) & ~63) * 2;
}

template <int ACT, int OUT, int TPW, bool PLAIN, int XM>
static hipError_t mp_launch(const MlpPArgs& a, size_t lds, hipStream_t st) {
  auto k = &mlp_persistent_kernel<ACT, OUT, TPW, PLAIN, XM>;
  static int lds_set = -1;  // per instantiation: the attribute call is host work on every launch otherwise
  if ((int)lds > lds_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    lds_set = (int)lds;
  }
  const int grid = XM == 3 ? 1 + a.nh : 1;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kMpThreads), lds, st, a);
  return hipGetLastError();
}

// Instantiated for the shapes this path serves (out = 1, H <= 512: the toy /
// 2-layer MLP configurations); wider heads or hidden layers spill registers here
// and run on the multi-workgroup kernel (csrc/mlp_fused.hip) instead.
template <int ACT>
static hipError_t mp_launch_out(const MlpPArgs& a, size_t lds, hipStream_t st) {
  if (a.out_dim != 1 || a.hidden > 512) return hipErrorInvalidValue;
  const bool plain = a.momentum == 0.f && a.weight_decay == 0.f && !a.maximize;
  if (a.world > 1) {
    switch (a.xmode) {
      case 1: return plain ? mp_launch<ACT, 1, 2, true, 1>(a, lds, st) : mp_launch<ACT, 1, 2, false, 1>(a, lds, st);
      case 2: return plain ? mp_launch<ACT, 1, 2, true, 2>(a, lds, st) : mp_launch<ACT, 1, 2, false, 2>(a, lds, st);
      case 3: return plain ? mp_launch<ACT, 1, 2, true, 3>(a, lds, st) : mp_launch<ACT, 1, 2, false, 3>(a, lds, st);
      default: return hipErrorInvalidValue;
    }
  }
  return plain ? mp_launch<ACT, 1, 2, true, 0>(a, lds, st) : mp_launch<ACT, 1, 2, false, 0>(a, lds, st);
}

hipError_t dta_mlp_persistent(const MlpPArgs* a, int act, hipStream_t st) {
  if (a->B < 1 || a->B > 32 || a->in_dim < 1 || a->in_dim + 1 + a->out_dim > kMpXs || a->hidden % 32 ||
      a->out_dim != 1 || a->hidden > 512 ||
      a->nsteps < 1)
    return hipErrorInvalidValue;
  // momenta live in LDS only with several ranks (one rank: in the owning lanes' registers)
  const size_t lds = dta_mlp_persistent_lds_bytes(a->total, a->hidden, a->out_dim, a->M != nullptr && a->world > 1);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  switch (act) {
    case ACT_NONE: return mp_launch_out<ACT_NONE>(*a, lds, st);
    case ACT_RELU: return mp_launch_out<ACT_RELU>(*a, lds, st);
    case ACT_GELU_TANH: return mp_launch_out<ACT_GELU_TANH>(*a, lds, st);
    case ACT_SILU: return mp_launch_out<ACT_SILU>(*a, lds, st);
    default: return hipErrorInvalidValue;
  }
}
