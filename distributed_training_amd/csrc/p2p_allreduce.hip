// One-shot intra-node all-reduce over xGMI peer memory (gfx950 / MI355X).
//
// Why: the headline configuration all-reduces
// a ~45 KB gradient bucket every ~10 us step.  A ring all-reduce of that size
// is pure latency (2(W-1) dependent hops); on xGMI every GPU has a direct link
// to every other GPU, so one "push" hop suffices: each rank writes its bucket
// straight into a slot of every peer's receive buffer (7 links in parallel),
// raises a flag in each peer, waits for the W-1 flags addressed to it, and
// sums the W slots locally in rank order -- so every rank computes bit-identical
// results.  One kernel launch, graph-capturable, no host involvement.
//
// Protocol (per workgroup w, which owns one contiguous chunk of the bucket):
//   epoch e = ++epoch_ctr (device counter, one value per call for all
//   workgroups: hipGraph replays advance it);
//   parity p = e & 1 selects one of two slot sets, so a slot is only rewritten
//   two epochs later, after every peer has signalled epoch e+1 -- which it does
//   only after it finished reading epoch e.
//   push    : peer[q].slot[p][rank][chunk] = data[chunk]     (q != rank)
//   release : __threadfence_system(); peer[q].flag[p][w][rank] = e
//   acquire : spin until local flag[p][w][q] == e for every q != rank (bounded:
//             on timeout an error flag is raised and the kernel exits, so a
//             dead peer can never hang the GPU)
//   reduce  : data[chunk] = scale * sum_q (q == rank ? data : slot[p][q])
// LL mode (default): every element travels as one 8-byte store {f32 bits,
// epoch} into the peer's slot, so no release fence, no flag and no extra
// round trip are needed: the receiver polls each element until its tag equals
// the epoch (slot reuse is safe by the same two-epoch argument: a rank only
// starts epoch e+2 after receiving every peer's epoch e+1 data, which each
// peer sends only after it finished reading epoch e).  Twice the bytes on the
// link, which is free at the bucket sizes this path is used for.
// The shared buffer is allocated uncached (hipDeviceMallocUncached, as RCCL's
// low-latency buffers are) so remote writes are never hidden behind stale L2
// lines, and exported with hipIpcGetMemHandle (dmabuf IPC).
#include "common.h"

#include <cstring>

namespace dta {

constexpr int kP2PMaxRanks = 8;
constexpr int kP2PMaxWG = 64;
constexpr int kP2PThreads = 512;

struct P2PArgs {
  float* data;
  int64_t n;
  int64_t chunk;           // elements per workgroup (multiple of 4)
  int64_t max_elems;       // slot capacity
  float scale;
  int rank, world;
  float* peer_data[kP2PMaxRanks];   // base of each rank's slot array [2][world][max_elems]
  int* peer_flags[kP2PMaxRanks];    // base of each rank's flags [2][kP2PMaxWG][world]
  int* local_flags;
  const float* local_data;          // == peer_data[rank]
  int* epoch_ctr;                   // [kP2PMaxWG], local, not shared
  int* err;
  int* err_host;                    // host-mapped copy of err: polled by the engines without a device sync
  int timeout_iters;
  uint64_t* peer_ll[kP2PMaxRanks];  // LL slots [2][world][max_elems] of {f32, epoch}
  const uint64_t* local_ll;
};

__device__ __forceinline__ bool peer_failed(int* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

__device__ __forceinline__ void raise_err(const P2PArgs& a) {
  atomicOr(a.err, 1);
  if (a.err_host) __hip_atomic_store(a.err_host, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The epoch is global per call: every workgroup slot counter advances together
// (workgroup 0 also advances the counters of workgroups this launch did not
// use), so element i alternates parity on every call even when consecutive
// calls split the buffer into different chunks -- otherwise a slot could be
// rewritten while a peer still reads it, or carry a stale tag that matches.
__device__ __forceinline__ void advance_epochs(const P2PArgs& a, int epoch) {
  if (threadIdx.x == 0) a.epoch_ctr[blockIdx.x] = epoch;
  if (blockIdx.x == 0)
    for (int x = gridDim.x + threadIdx.x; x < kP2PMaxWG; x += blockDim.x) a.epoch_ctr[x] = epoch;
}

__global__ void __launch_bounds__(kP2PThreads) p2p_allreduce_ll_kernel(P2PArgs a) {
  const int w = blockIdx.x, tid = threadIdx.x;
  const int64_t c0 = (int64_t)w * a.chunk;
  const int64_t c1 = min(c0 + a.chunk, a.n);
  const unsigned epoch = (unsigned)a.epoch_ctr[w] + 1u;
  const int par = epoch & 1;
  const int W = a.world;
  // push: {value, epoch} into slot [par][rank] of every peer
  for (int64_t i = c0 + tid; i < c1; i += kP2PThreads) {
    const uint64_t v = (uint64_t)__float_as_uint(a.data[i]) | ((uint64_t)epoch << 32);
    for (int q = 0; q < W; ++q) {
      if (q == a.rank) continue;
      __hip_atomic_store(a.peer_ll[q] + ((int64_t)par * W + a.rank) * a.max_elems + i, v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  // receive + reduce in rank order
  for (int64_t i = c0 + tid; i < c1; i += kP2PThreads) {
    float acc = 0.f;
    for (int q = 0; q < W; ++q) {
      if (q == a.rank) {
        acc += a.data[i];
        continue;
      }
      const uint64_t* src = a.local_ll + ((int64_t)par * W + q) * a.max_elems + i;
      uint64_t v = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      int it = 0;
      while ((unsigned)(v >> 32) != epoch) {
        // bounded wait; once any wait timed out (sticky error flag) every later
        // wait gives up at once, so a dead peer costs one timeout, not one per element
        if (++it > a.timeout_iters || ((it & 1023) == 1 && peer_failed(a.err))) {
          raise_err(a);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        v = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      acc += __uint_as_float((unsigned)(v & 0xffffffffu));
    }
    a.data[i] = acc * a.scale;
  }
  __syncthreads();
  advance_epochs(a, (int)epoch);
}

__global__ void __launch_bounds__(kP2PThreads) p2p_allreduce_kernel(P2PArgs a) {
  const int w = blockIdx.x, tid = threadIdx.x;
  const int64_t c0 = (int64_t)w * a.chunk;
  const int64_t c1 = min(c0 + a.chunk, a.n);
  const int epoch = a.epoch_ctr[w] + 1;
  const int par = epoch & 1;
  const int W = a.world;
  const int64_t v0 = c0 >> 2, v1 = c1 >> 2;  // float4 range (c0 % 4 == 0)
  const bool tail = (c1 == a.n) && (a.n & 3);
  // ---- push my chunk into every peer's slot [par][rank] ----
  for (int q = 0; q < W; ++q) {
    if (q == a.rank) continue;
    float* dst = a.peer_data[q] + ((int64_t)par * W + a.rank) * a.max_elems;
    for (int64_t i = v0 + tid; i < v1; i += kP2PThreads)
      reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(a.data)[i];
    if (tail)
      for (int64_t i = (v1 << 2) + tid; i < c1; i += kP2PThreads) dst[i] = a.data[i];
  }
  __threadfence_system();
  __syncthreads();
  // ---- release: flag[par][w][rank] = epoch in every peer ----
  if (tid < W && tid != a.rank)
    __hip_atomic_store(a.peer_flags[tid] + ((int64_t)par * kP2PMaxWG + w) * W + a.rank, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  // ---- acquire: wait for every peer's flag for (par, w) ----
  if (tid < W && tid != a.rank) {
    const int* f = a.local_flags + ((int64_t)par * kP2PMaxWG + w) * W + tid;
    int it = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      if (++it > a.timeout_iters || ((it & 1023) == 1 && peer_failed(a.err))) {
        raise_err(a);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  // ---- reduce in rank order (identical on every rank) ----
  for (int64_t i = v0 + tid; i < v1; i += kP2PThreads) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = 0; q < W; ++q) {
      const float4 v = q == a.rank ? reinterpret_cast<const float4*>(a.data)[i]
                                   : reinterpret_cast<const float4*>(a.local_data +
                                                                     ((int64_t)par * W + q) * a.max_elems)[i];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    acc.x *= a.scale;
    acc.y *= a.scale;
    acc.z *= a.scale;
    acc.w *= a.scale;
    reinterpret_cast<float4*>(a.data)[i] = acc;
  }
  if (tail)
    for (int64_t i = (v1 << 2) + tid; i < c1; i += kP2PThreads) {
      float acc = 0.f;
      for (int q = 0; q < W; ++q)
        acc += q == a.rank ? a.data[i] : a.local_data[((int64_t)par * W + q) * a.max_elems + i];
      a.data[i] = acc * a.scale;
    }
  advance_epochs(a, epoch);
}

struct P2PState {
  int rank = 0, world = 1;
  int64_t max_elems = 0;
  char* buf = nullptr;  // shared: slots [2][world][max_elems] f32, flags [2][kP2PMaxWG][world] i32, LL slots
  size_t flags_off = 0, ll_off = 0, bytes = 0;
  int ll = 1;
  int* epoch = nullptr;
  int* err = nullptr;
  int* err_host = nullptr;
  char* peers[kP2PMaxRanks] = {};
  bool opened = false;
};

}  // namespace dta

using namespace dta;

// handle_out: 64-byte hipIpcMemHandle_t of the shared buffer
hipError_t dta_p2p_create(int rank, int world, int64_t max_elems, void** state_out, void* handle_out) {
  if (world < 1 || world > kP2PMaxRanks || rank < 0 || rank >= world || max_elems <= 0) return hipErrorInvalidValue;
  auto* s = new P2PState();
  s->rank = rank;
  s->world = world;
  s->max_elems = (max_elems + 3) / 4 * 4;
  s->flags_off = ((size_t)2 * world * s->max_elems * sizeof(float) + 4095) / 4096 * 4096;
  s->ll_off = (s->flags_off + (size_t)2 * kP2PMaxWG * world * sizeof(int) + 4095) / 4096 * 4096;
  s->bytes = s->ll_off + (size_t)2 * world * s->max_elems * sizeof(uint64_t);
  hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&s->buf), s->bytes, hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(s->buf, 0, s->bytes);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s->epoch), kP2PMaxWG * sizeof(int) + 64);
  if (e == hipSuccess) e = hipMemset(s->epoch, 0, kP2PMaxWG * sizeof(int) + 64);
  if (e == hipSuccess) s->err = s->epoch + kP2PMaxWG;
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void**>(&s->err_host), 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) *s->err_host = 0;
  hipIpcMemHandle_t h;
  if (e == hipSuccess) e = hipIpcGetMemHandle(&h, s->buf);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    if (s->buf) (void)hipFree(s->buf);
    if (s->epoch) (void)hipFree(s->epoch);
    if (s->err_host) (void)hipHostFree(s->err_host);
    delete s;
    return e;
  }
  std::memcpy(handle_out, &h, sizeof(h));
  s->peers[rank] = s->buf;
  *state_out = s;
  return hipSuccess;
}

int dta_p2p_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

// handles: world x 64 bytes (this rank's entry is ignored)
hipError_t dta_p2p_open(void* state, const void* handles) {
  auto* s = static_cast<P2PState*>(state);
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

// LL slot arrays of every rank (for kernels that exchange through them directly,
// e.g. the persistent MLP loop), the error flag and a spare device counter.
hipError_t dta_p2p_ll_info(void* state, unsigned long long* peer_ll, unsigned long long* local_ll, int* rank,
                           int* world, long long* slot_elems, unsigned long long* err, unsigned long long* counter) {
  auto* s = static_cast<P2PState*>(state);
  if (!s->opened) return hipErrorInvalidValue;
  for (int q = 0; q < s->world; ++q) peer_ll[q] = reinterpret_cast<unsigned long long>(s->peers[q] + s->ll_off);
  *local_ll = reinterpret_cast<unsigned long long>(s->buf + s->ll_off);
  *rank = s->rank;
  *world = s->world;
  *slot_elems = s->max_elems;
  *err = reinterpret_cast<unsigned long long>(s->err);
  *counter = reinterpret_cast<unsigned long long>(s->epoch + kP2PMaxWG + 1);  // after err: a free int
  return hipSuccess;
}

// This rank's uncached (fine-grained, MTYPE UC) data and flag regions, for
// kernels that hand data between workgroups of one GPU through them with plain
// stores + s_waitcnt + relaxed flag atomics (no L2 write-back / invalidate):
// the persistent MLP loop's helper exchange.  Unused by the LL protocol.
hipError_t dta_p2p_regions(void* state, unsigned long long* data, long long* data_bytes, unsigned long long* flags,
                           long long* flags_bytes) {
  auto* s = static_cast<P2PState*>(state);
  *data = reinterpret_cast<unsigned long long>(s->buf);
  *data_bytes = (long long)2 * s->world * s->max_elems * (long long)sizeof(float);
  *flags = reinterpret_cast<unsigned long long>(s->buf + s->flags_off);
  *flags_bytes = (long long)2 * kP2PMaxWG * s->world * (long long)sizeof(int);
  return hipSuccess;
}

int dta_p2p_num_wg(int64_t n) {
  // ~2048 elements (8 KiB) per workgroup: enough memory-level parallelism per
  // link without spreading a 45 KB bucket over more flag round trips
  int64_t g = (n + 2047) / 2048;
  return (int)(g < 1 ? 1 : (g > kP2PMaxWG ? kP2PMaxWG : g));
}

void dta_p2p_set_ll(void* state, int ll) { static_cast<P2PState*>(state)->ll = ll; }

hipError_t dta_p2p_allreduce(void* state, float* data, int64_t n, float scale, int timeout_iters, hipStream_t st) {
  auto* s = static_cast<P2PState*>(state);
  if (!s->opened || n <= 0 || n > s->max_elems || (reinterpret_cast<uintptr_t>(data) & 15)) return hipErrorInvalidValue;
  P2PArgs a{};
  a.data = data;
  a.n = n;
  const int nwg = dta_p2p_num_wg(n);
  a.chunk = ((n + nwg - 1) / nwg + 3) / 4 * 4;
  a.max_elems = s->max_elems;
  a.scale = scale;
  a.rank = s->rank;
  a.world = s->world;
  for (int q = 0; q < s->world; ++q) {
    a.peer_data[q] = reinterpret_cast<float*>(s->peers[q]);
    a.peer_flags[q] = reinterpret_cast<int*>(s->peers[q] + s->flags_off);
    a.peer_ll[q] = reinterpret_cast<uint64_t*>(s->peers[q] + s->ll_off);
  }
  a.local_ll = reinterpret_cast<const uint64_t*>(s->buf + s->ll_off);
  a.local_flags = reinterpret_cast<int*>(s->buf + s->flags_off);
  a.local_data = reinterpret_cast<const float*>(s->buf);
  a.epoch_ctr = s->epoch;
  a.err = s->err;
  a.err_host = s->err_host;
  a.timeout_iters = timeout_iters;
  const int grid = (int)((n + a.chunk - 1) / a.chunk);
  if (s->ll) hipLaunchKernelGGL(p2p_allreduce_ll_kernel, dim3(grid), dim3(kP2PThreads), 0, st, a);
  else hipLaunchKernelGGL(p2p_allreduce_kernel, dim3(grid), dim3(kP2PThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t dta_p2p_error(void* state, int* out) {
  auto* s = static_cast<P2PState*>(state);
  return hipMemcpy(out, s->err, sizeof(int), hipMemcpyDeviceToHost);
}

// The all-reduce kernels' timeout flag as seen by the host, without a device sync
// (the persistent MLP loop raises only the device flag: dta_p2p_error covers it).
int dta_p2p_error_nosync(void* state) {
  return __atomic_load_n(static_cast<P2PState*>(state)->err_host, __ATOMIC_ACQUIRE);
}

// Re-arm after a timed-out exchange that was expected to be survivable (e.g. a
// probe of an exchange form during calibration); every rank clears together.
hipError_t dta_p2p_clear_error(void* state) {
  auto* s = static_cast<P2PState*>(state);
  __atomic_store_n(s->err_host, 0, __ATOMIC_RELEASE);
  return hipMemset(s->err, 0, sizeof(int));
}

void dta_p2p_destroy(void* state) {
  auto* s = static_cast<P2PState*>(state);
  if (!s) return;
  (void)hipDeviceSynchronize();
  for (int q = 0; q < s->world; ++q)
    if (q != s->rank && s->peers[q]) (void)hipIpcCloseMemHandle(s->peers[q]);
  if (s->buf) (void)hipFree(s->buf);
  if (s->epoch) (void)hipFree(s->epoch);
  if (s->err_host) (void)hipHostFree(s->err_host);
  delete s;
}
