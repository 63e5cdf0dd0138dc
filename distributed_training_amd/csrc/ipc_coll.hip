// Intra-node collectives over IPC-mapped peer memory (gfx950 / MI355X).
//
// What: all-reduce, reduce-scatter, all-gather and broadcast of fp32 / bf16
// tensors between the ranks of one node, each ONE kernel launch on the
// caller's stream (graph-capturable, no host involvement), for the DDP
// gradient buckets and the FSDP unit gathers / scatters (SURVEY.md §2.7 X3,
// X5, X6; §5.8).
//
// Why not a ring: xGMI is point-to-point -- every MI355X has a direct link to
// each of its 7 peers.  A ring uses one of them per step and needs 2(W-1)
// dependent steps.  Here every transfer is a direct push over its own link,
// all 7 links at once:
//   all-reduce (two-shot): each rank pushes chunk q of its tensor into rank q's
//     receive slot (W-1 links in parallel); rank q sums chunk q over the W
//     contributions IN RANK ORDER (fp32 accumulation, one rounding) and pushes
//     the sum to every rank's gather slot; everyone copies the W sums out.
//     2 hops of latency for any W, (W-1)/W of the tensor on each link each
//     way, and every rank ends with bit-identical values (each chunk is
//     reduced exactly once, by its owner).
//   reduce-scatter: the first half of that; all-gather: the second half
//     (each rank pushes its shard); broadcast: the source pushes to all.
//
// Protocol (per workgroup w, which owns the same sub-range of every chunk on
// every rank): epoch e = ++ctr[w] (device counter: graph replays advance it),
// parity p = e & 1 selects one of two slot sets.  A producer stores its data
// into the peer's slot with plain 16-byte stores, then system-scope release
// (fence + flag store) of flag[p][w][me] = e in the peer; a consumer waits
// (system-scope acquire) for flag[p][w][q] == e of every peer q before it
// reads.  EVERY operation makes every rank receive a flag from every other
// rank in every epoch (the broadcast's receivers signal too), so no rank can
// start epoch e + 2 -- and rewrite a parity-p slot -- before every peer has
// finished reading epoch e.
// Waits are bounded in wall time (s_memrealtime): on timeout a sticky error
// is raised in device memory AND in host-mapped memory (the engines poll the
// host copy every step without a device sync) and the kernel exits, so a dead
// peer can never hang the GPU.
// Slots and flags live in uncached device memory (hipDeviceMallocUncached, as
// RCCL's own low-latency buffers), exported by dmabuf IPC: a remote store is
// never hidden behind a stale L2 line of the receiver.
#include "common.h"

#include <cstring>

namespace dta {

constexpr int kIpcMaxRanks = 8;
constexpr int kIpcMaxWG = 128;
constexpr int kIpcThreads = 512;

enum IpcOp : int { IPC_ALLREDUCE = 0, IPC_REDUCE_SCATTER = 1, IPC_ALLGATHER = 2, IPC_BROADCAST = 3 };
enum IpcRed : int { RED_SUM = 0, RED_MAX = 1, RED_MIN = 2 };

struct IpcArgs {
  char* data;          // AR / BC: in-out; RS: out [m]; AG: out [W m]
  const char* src;     // RS: in [W m]; AG: in [m]; unused otherwise
  int64_t n;           // AR: elements of data; BC: elements; RS / AG: m
  int64_t m;           // chunk elements (AR: ceil(n / W) rounded to 8)
  int64_t cstride;     // bytes between consecutive chunks of the W-chunk tensor (AR data, RS src, AG data)
  int esize;           // bytes per element (AR / RS: 4 = fp32, 2 = bf16)
  int red;             // IpcRed
  float scale;         // applied to reduced values (1/W for avg)
  int rank, world, root;
  int nwg;
  int64_t slot_bytes;  // one slot (one source rank, one parity)
  char* peer_rs[kIpcMaxRanks];  // each rank's receive-slot region [2][W][slot_bytes]
  char* peer_ag[kIpcMaxRanks];  // each rank's gather-slot region  [2][W][slot_bytes]
  int* peer_rsf[kIpcMaxRanks];  // each rank's flags [2][kIpcMaxWG][W]
  int* peer_agf[kIpcMaxRanks];
  int* ctr;            // [kIpcMaxWG] local epoch counters
  int* err;            // device sticky error
  int* err_host;       // host-mapped copy of the error (polled without a device sync)
  long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
};

__device__ __forceinline__ bool ipc_failed(const IpcArgs& a) {
  return __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

__device__ __forceinline__ void ipc_raise(const IpcArgs& a) {
  __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.err_host) __hip_atomic_store(a.err_host, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// signal every peer (thread q < W, q != rank), after this workgroup's stores
__device__ __forceinline__ void ipc_signal(const IpcArgs& a, int* const* peer_flags, int par, int w, int ep) {
  __threadfence_system();
  __syncthreads();
  const int q = threadIdx.x;
  if (q < a.world && q != a.rank)
    __hip_atomic_store(peer_flags[q] + ((int64_t)par * kIpcMaxWG + w) * a.world + a.rank, ep, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// wait for the flag of every peer (bounded); the whole workgroup leaves together
__device__ __forceinline__ void ipc_wait(const IpcArgs& a, int* my_flags, int par, int w, int ep) {
  const int q = threadIdx.x;
  if (q < a.world && q != a.rank) {
    const int* f = my_flags + ((int64_t)par * kIpcMaxWG + w) * a.world + q;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    int it = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != ep) {
      if ((++it & 255) == 0) {
        if (ipc_failed(a) || (long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
          ipc_raise(a);
          break;
        }
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
}

__device__ __forceinline__ void ipc_advance(const IpcArgs& a, int ep) {
  __syncthreads();
  if (threadIdx.x == 0) a.ctr[blockIdx.x] = ep;
  if (blockIdx.x == 0)
    for (int x = gridDim.x + threadIdx.x; x < kIpcMaxWG; x += blockDim.x) a.ctr[x] = ep;
}

// ---- 16-byte vectors of 8 (bf16) or 4 (fp32) elements ----
__device__ __forceinline__ uint4 ld16(const char* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ void st16(char* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }

// byte range [b0, b1) of one chunk handled by workgroup w: whole 16-B vectors,
// split evenly over the workgroups (the last one also takes the tail bytes)
struct Range {
  int64_t b0, b1;
};
__device__ __forceinline__ Range wg_range(int64_t chunk_bytes, int w, int nwg) {
  const int64_t nv = chunk_bytes >> 4;
  const int64_t per = (nv + nwg - 1) / nwg;
  int64_t v0 = (int64_t)w * per, v1 = v0 + per;
  if (v0 > nv) v0 = nv;
  if (v1 > nv) v1 = nv;
  Range r{v0 << 4, v1 << 4};
  if (w == nwg - 1) r.b1 = chunk_bytes;  // tail (< 16 bytes) by 2-byte copies
  return r;
}

__device__ __forceinline__ void copy_range(char* dst, const char* src, Range r) {
  const int64_t vend = r.b1 & ~(int64_t)15;
  for (int64_t b = r.b0 + 16 * (int64_t)threadIdx.x; b < vend; b += 16 * kIpcThreads) st16(dst + b, ld16(src + b));
  for (int64_t b = (vend > r.b0 ? vend : r.b0) + 2 * (int64_t)threadIdx.x; b < r.b1; b += 2 * kIpcThreads)
    *reinterpret_cast<unsigned short*>(dst + b) = *reinterpret_cast<const unsigned short*>(src + b);
}

// all-reduce chunk q of data: elements [q m, min(n, (q+1) m))
__device__ __forceinline__ int64_t chunk_elems(const IpcArgs& a, int q) {
  const int64_t s = (int64_t)q * a.m;
  const int64_t e = s + a.m < a.n ? s + a.m : a.n;
  return e > s ? e - s : 0;
}

template <typename T>
__device__ __forceinline__ void unpack16(uint4 v, float* f);
template <>
__device__ __forceinline__ void unpack16<float>(uint4 v, float* f) {
  f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y); f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
}
template <>
__device__ __forceinline__ void unpack16<bf16>(uint4 v, float* f) {
  const bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = bf2f(b[j]);
}
template <typename T>
__device__ __forceinline__ uint4 pack16(const float* f);
template <>
__device__ __forceinline__ uint4 pack16<float>(const float* f) {
  return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
}
template <>
__device__ __forceinline__ uint4 pack16<bf16>(const float* f) {
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = f2bf(f[j]);
  return __builtin_bit_cast(uint4, b);
}

__device__ __forceinline__ float red_op(int red, float x, float y) {
  return red == RED_SUM ? x + y : (red == RED_MAX ? fmaxf(x, y) : fminf(x, y));
}

// Reduce the byte range r of this rank's chunk over all ranks in rank order:
// own contribution at `own`, rank q's at my receive slot q.  Result (scaled)
// written to `out` and, when `push`, to every peer's gather slot [par][me].
template <typename T>
__device__ void reduce_range(const IpcArgs& a, const char* own, char* out, int par, Range r, bool push) {
  constexpr int E = 16 / sizeof(T);
  const char* my_rs = a.peer_rs[a.rank];
  const int64_t vend = r.b1 & ~(int64_t)15;
  for (int64_t b = r.b0 + 16 * (int64_t)threadIdx.x; b < vend; b += 16 * kIpcThreads) {
    float acc[E], x[E];
    for (int q = 0; q < a.world; ++q) {
      const char* p = q == a.rank ? own + b : my_rs + ((int64_t)par * a.world + q) * a.slot_bytes + b;
      unpack16<T>(ld16(p), x);
#pragma unroll
      for (int j = 0; j < E; ++j) acc[j] = q == 0 ? x[j] : red_op(a.red, acc[j], x[j]);
    }
#pragma unroll
    for (int j = 0; j < E; ++j) acc[j] *= a.scale;
    const uint4 v = pack16<T>(acc);
    st16(out + b, v);
    if (push)
      for (int q = 0; q < a.world; ++q)
        if (q != a.rank) st16(a.peer_ag[q] + ((int64_t)par * a.world + a.rank) * a.slot_bytes + b, v);
  }
  // tail elements (fewer than one vector), one per thread
  for (int64_t b = (vend > r.b0 ? vend : r.b0) + (int64_t)sizeof(T) * threadIdx.x; b < r.b1;
       b += (int64_t)sizeof(T) * kIpcThreads) {
    float acc = 0.f;
    for (int q = 0; q < a.world; ++q) {
      const char* p = q == a.rank ? own + b : my_rs + ((int64_t)par * a.world + q) * a.slot_bytes + b;
      const float x = (float)*reinterpret_cast<const T*>(p);
      acc = q == 0 ? x : red_op(a.red, acc, x);
    }
    const T v = (T)(acc * a.scale);
    *reinterpret_cast<T*>(out + b) = v;
    if (push)
      for (int q = 0; q < a.world; ++q)
        if (q != a.rank) *reinterpret_cast<T*>(a.peer_ag[q] + ((int64_t)par * a.world + a.rank) * a.slot_bytes + b) = v;
  }
}

template <typename T, int OP>
__global__ void __launch_bounds__(kIpcThreads) ipc_coll_kernel(IpcArgs a) {
  const int w = blockIdx.x;
  const int ep = a.ctr[w] + 1;
  const int par = ep & 1;
  const int W = a.world, me = a.rank;
  const int64_t es = sizeof(T);
  if constexpr (OP == IPC_ALLREDUCE || OP == IPC_REDUCE_SCATTER) {
    // phase 1: chunk q of the input -> rank q's receive slot [par][me]
    const char* in = OP == IPC_ALLREDUCE ? a.data : a.src;
    for (int q = 0; q < W; ++q) {
      if (q == me) continue;
      const int64_t cb = (OP == IPC_ALLREDUCE ? chunk_elems(a, q) : a.m) * es;
      const Range r = wg_range(cb, w, a.nwg);
      copy_range(a.peer_rs[q] + ((int64_t)par * W + me) * a.slot_bytes, in + (int64_t)q * a.cstride, r);
    }
    ipc_signal(a, a.peer_rsf, par, w, ep);
    ipc_wait(a, a.peer_rsf[me], par, w, ep);
    // phase 2: reduce my chunk in rank order
    const int64_t cb = (OP == IPC_ALLREDUCE ? chunk_elems(a, me) : a.m) * es;
    const Range r = wg_range(cb, w, a.nwg);
    const char* own = in + (int64_t)me * a.cstride;
    char* out = OP == IPC_ALLREDUCE ? a.data + (int64_t)me * a.cstride : a.data;
    reduce_range<T>(a, own, out, par, r, OP == IPC_ALLREDUCE);
    if constexpr (OP == IPC_ALLREDUCE) {
      // phase 3: every rank's sum of its chunk -> my tensor
      ipc_signal(a, a.peer_agf, par, w, ep);
      ipc_wait(a, a.peer_agf[me], par, w, ep);
      for (int q = 0; q < W; ++q) {
        if (q == me) continue;
        const Range rq = wg_range(chunk_elems(a, q) * es, w, a.nwg);
        copy_range(a.data + (int64_t)q * a.cstride, a.peer_ag[me] + ((int64_t)par * W + q) * a.slot_bytes, rq);
      }
    }
  } else if constexpr (OP == IPC_ALLGATHER) {
    const Range r = wg_range(a.m * es, w, a.nwg);
    for (int q = 0; q < W; ++q)
      if (q != me) copy_range(a.peer_ag[q] + ((int64_t)par * W + me) * a.slot_bytes, a.src, r);
    if (a.data + (int64_t)me * a.cstride != a.src) copy_range(a.data + (int64_t)me * a.cstride, a.src, r);
    ipc_signal(a, a.peer_agf, par, w, ep);
    ipc_wait(a, a.peer_agf[me], par, w, ep);
    for (int q = 0; q < W; ++q)
      if (q != me) copy_range(a.data + (int64_t)q * a.cstride, a.peer_ag[me] + ((int64_t)par * W + q) * a.slot_bytes, r);
  } else {  // broadcast from a.root
    const Range r = wg_range(a.n * es, w, a.nwg);
    if (me == a.root)
      for (int q = 0; q < W; ++q)
        if (q != me) copy_range(a.peer_ag[q] + ((int64_t)par * W + me) * a.slot_bytes, a.data, r);
    ipc_signal(a, a.peer_agf, par, w, ep);  // receivers signal too (slot-reuse guarantee)
    ipc_wait(a, a.peer_agf[me], par, w, ep);
    if (me != a.root) copy_range(a.data, a.peer_ag[me] + ((int64_t)par * W + a.root) * a.slot_bytes, r);
  }
  ipc_advance(a, ep);
}

struct IpcState {
  int rank = 0, world = 1;
  int64_t slot_bytes = 0;
  char* buf = nullptr;  // [rs: 2 W slot][ag: 2 W slot][rs flags][ag flags]
  size_t ag_off = 0, rsf_off = 0, agf_off = 0, bytes = 0;
  int* ctr = nullptr;   // [kIpcMaxWG] counters + err
  int* err = nullptr;
  int* err_host = nullptr;
  char* peers[kIpcMaxRanks] = {};
  bool opened = false;
};

}  // namespace dta

using namespace dta;

hipError_t dta_ipc_create(int rank, int world, int64_t slot_bytes, void** state_out, void* handle_out) {
  if (world < 1 || world > kIpcMaxRanks || rank < 0 || rank >= world || slot_bytes <= 0) return hipErrorInvalidValue;
  auto* s = new IpcState();
  s->rank = rank;
  s->world = world;
  s->slot_bytes = (slot_bytes + 255) / 256 * 256;
  const size_t region = (size_t)2 * world * s->slot_bytes;
  const size_t flags = (size_t)2 * kIpcMaxWG * world * sizeof(int);
  s->ag_off = region;
  s->rsf_off = 2 * region;
  s->agf_off = (s->rsf_off + flags + 255) / 256 * 256;
  s->bytes = (s->agf_off + flags + 4095) / 4096 * 4096;
  hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&s->buf), s->bytes, hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(s->buf + s->rsf_off, 0, s->bytes - s->rsf_off);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s->ctr), (kIpcMaxWG + 16) * sizeof(int));
  if (e == hipSuccess) e = hipMemset(s->ctr, 0, (kIpcMaxWG + 16) * sizeof(int));
  if (e == hipSuccess) s->err = s->ctr + kIpcMaxWG;
  if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s->err_host), 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) *s->err_host = 0;
  hipIpcMemHandle_t h;
  if (e == hipSuccess) e = hipIpcGetMemHandle(&h, s->buf);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    if (s->buf) (void)hipFree(s->buf);
    if (s->ctr) (void)hipFree(s->ctr);
    if (s->err_host) (void)hipHostFree(s->err_host);
    delete s;
    return e;
  }
  std::memcpy(handle_out, &h, sizeof(h));
  s->peers[rank] = s->buf;
  *state_out = s;
  return hipSuccess;
}

int dta_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

hipError_t dta_ipc_open(void* state, const void* handles) {
  auto* s = static_cast<IpcState*>(state);
  for (int q = 0; q < s->world; ++q) {
    if (q == s->rank) continue;
    hipIpcMemHandle_t h;
    std::memcpy(&h, static_cast<const char*>(handles) + (size_t)q * sizeof(h), sizeof(h));
    void* p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return e;
    s->peers[q] = static_cast<char*>(p);
  }
  s->opened = true;
  return hipSuccess;
}

int64_t dta_ipc_slot_bytes(void* state) { return static_cast<IpcState*>(state)->slot_bytes; }

// one launch: op (IpcOp), dtype_bytes (4 fp32 / 2 bf16; movement ops: any even size),
// n / m as in IpcArgs; the caller has checked alignment (16 B) and capacity
hipError_t dta_ipc_launch(void* state, int op, int dtype_bytes, int red, float scale, void* data, const void* src,
                          int64_t n, int64_t m, int64_t cstride, int root, double timeout_s, hipStream_t st) {
  auto* s = static_cast<IpcState*>(state);
  if (!s->opened || n < 0 || m < 0) return hipErrorInvalidValue;
  IpcArgs a{};
  a.data = static_cast<char*>(data);
  a.src = static_cast<const char*>(src);
  a.n = n;
  a.m = m;
  a.cstride = cstride;
  a.esize = dtype_bytes;
  a.red = red;
  a.scale = scale;
  a.rank = s->rank;
  a.world = s->world;
  a.root = root;
  a.slot_bytes = s->slot_bytes;
  for (int q = 0; q < s->world; ++q) {
    a.peer_rs[q] = s->peers[q];
    a.peer_ag[q] = s->peers[q] + s->ag_off;
    a.peer_rsf[q] = reinterpret_cast<int*>(s->peers[q] + s->rsf_off);
    a.peer_agf[q] = reinterpret_cast<int*>(s->peers[q] + s->agf_off);
  }
  a.ctr = s->ctr;
  a.err = s->err;
  a.err_host = s->err_host;
  a.timeout_ticks = (long long)(timeout_s * 1e8);
  // bytes each workgroup moves per chunk: ~64 KiB per workgroup, 1 .. kIpcMaxWG
  const int64_t chunk_bytes = (op == IPC_BROADCAST ? n : m) * dtype_bytes;
  if (chunk_bytes > s->slot_bytes) return hipErrorInvalidValue;
  int64_t g = (chunk_bytes + 65535) / 65536;
  a.nwg = (int)(g < 1 ? 1 : (g > kIpcMaxWG ? kIpcMaxWG : g));
  const dim3 grid(a.nwg), block(kIpcThreads);
#define IPC_LAUNCH(T, OPV) hipLaunchKernelGGL((ipc_coll_kernel<T, OPV>), grid, block, 0, st, a)
  const bool f32 = dtype_bytes == 4;
  switch (op) {
    case IPC_ALLREDUCE:
      a.src = nullptr;
      if (f32) IPC_LAUNCH(float, IPC_ALLREDUCE); else if (dtype_bytes == 2) IPC_LAUNCH(bf16, IPC_ALLREDUCE);
      else return hipErrorInvalidValue;
      break;
    case IPC_REDUCE_SCATTER:
      if (!src) return hipErrorInvalidValue;
      if (f32) IPC_LAUNCH(float, IPC_REDUCE_SCATTER); else if (dtype_bytes == 2) IPC_LAUNCH(bf16, IPC_REDUCE_SCATTER);
      else return hipErrorInvalidValue;
      break;
    case IPC_ALLGATHER:
      if (!src) return hipErrorInvalidValue;
      IPC_LAUNCH(unsigned short, IPC_ALLGATHER);  // pure data movement: element size irrelevant (m in bytes / 2)
      break;
    case IPC_BROADCAST:
      a.src = nullptr;
      IPC_LAUNCH(unsigned short, IPC_BROADCAST);
      break;
    default: return hipErrorInvalidValue;
  }
#undef IPC_LAUNCH
  return hipGetLastError();
}

int dta_ipc_error(void* state) {
  auto* s = static_cast<IpcState*>(state);
  return __atomic_load_n(s->err_host, __ATOMIC_ACQUIRE);
}

hipError_t dta_ipc_clear_error(void* state) {
  auto* s = static_cast<IpcState*>(state);
  __atomic_store_n(s->err_host, 0, __ATOMIC_RELEASE);
  return hipMemset(s->err, 0, sizeof(int));
}

void dta_ipc_destroy(void* state) {
  auto* s = static_cast<IpcState*>(state);
  if (!s) return;
  (void)hipDeviceSynchronize();
  for (int q = 0; q < s->world; ++q)
    if (q != s->rank && s->peers[q]) (void)hipIpcCloseMemHandle(s->peers[q]);
  if (s->buf) (void)hipFree(s->buf);
  if (s->ctr) (void)hipFree(s->ctr);
  if (s->err_host) (void)hipHostFree(s->err_host);
  delete s;
}
