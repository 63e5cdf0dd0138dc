// Stable sort of a token-id vector with its source positions in ONE workgroup -- the grouping the
// embedding backward's sorted-run kernel (lm_ops.hip embedding_bwd_kernel) consumes.
//
// torch.sort(stable=True) of GPT-2's 8192 token ids ran as 6-8 launches per step (rocprim's block sort,
// three odd-even merge passes, transforms, an index fill and copies: ~55 us, profiles/
// gpt2_ddp_1gpu_kernels_r6y.txt).  Here 1024 threads hold the whole vector (8 or 16 ids each, blocked:
// thread t owns positions [t * IPT, (t + 1) * IPT)) and rocprim's block radix sort ranks it in LDS over
// only the id bits in use (16 for a 50304-token vocabulary: two 8-bit passes).  An LSD radix sort keeps
// equal keys in position order, so the result is torch.sort(stable=True)'s: sid ascending, perm the
// source positions of each run in increasing order (tests/test_lm_ops_gpu.py::test_sort_ids_matches_torch).
// Ids outside [0, V) take the key 2^bits - 1 >= V: they sort to the end and the run kernel skips them.
// Reference: the token embedding of the GPT-2 configs (nn.Embedding backward).
#include "common.h"

#include <rocprim/block/block_radix_sort.hpp>

namespace dta {

constexpr int kSortThreads = 1024;

template <int IPT>
__global__ void __launch_bounds__(kSortThreads) sort_ids_kernel(const int64_t* __restrict__ ids, int T, int64_t V,
                                                                int bits, int64_t* __restrict__ sid,
                                                                int64_t* __restrict__ perm) {
  using Sort = rocprim::block_radix_sort<unsigned, kSortThreads, IPT, unsigned>;
  __shared__ typename Sort::storage_type st;
  const unsigned pad = (1u << bits) - 1u;
  unsigned k[IPT], v[IPT];
  const int p0 = threadIdx.x * IPT;
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const int p = p0 + i;
    const int64_t id = p < T ? ids[p] : -1;
    k[i] = id >= 0 && id < V ? (unsigned)id : pad;
    v[i] = (unsigned)p;
  }
  Sort().sort(k, v, st, 0u, (unsigned)bits);
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const int p = p0 + i;
    if (p < T) {
      sid[p] = k[i] == pad ? V : (int64_t)k[i];  // (an out-of-range id: V, which the run kernel skips)
      perm[p] = v[i];
    }
  }
}

}  // namespace dta

int dta_sort_ids_max() { return 16 * dta::kSortThreads; }

// ids: T int64 token ids; sid / perm: T int64 outputs.  T <= dta_sort_ids_max(), 1 <= V < 2^31.
hipError_t dta_sort_ids(const int64_t* ids, int T, int64_t V, int64_t* sid, int64_t* perm, hipStream_t st) {
  if (T < 1 || T > dta_sort_ids_max() || V < 1 || V >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  int bits = 1;
  while (((int64_t)1 << bits) - 1 < V) ++bits;  // 2^bits - 1 >= V: the out-of-range key lies above every id
  if (T <= 8 * dta::kSortThreads)
    hipLaunchKernelGGL(dta::sort_ids_kernel<8>, dim3(1), dim3(dta::kSortThreads), 0, st, ids, T, V, bits, sid, perm);
  else
    hipLaunchKernelGGL(dta::sort_ids_kernel<16>, dim3(1), dim3(dta::kSortThreads), 0, st, ids, T, V, bits, sid, perm);
  return hipGetLastError();
}
