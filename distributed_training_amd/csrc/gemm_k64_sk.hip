// Stream-K instantiations of the 64-deep-stage GEMM (csrc/gemm_k64_kernels.h SkArgs): a translation unit of
// their own so they compile in parallel with csrc/gemm_k64.hip.
#include "gemm_k64_kernels.h"

using namespace dta;

hipError_t dta_gemm_k64_sk_launch(const k64::Args& g, const k64::SkArgs& s, int grid, int base, bool a_t, bool b_t,
                                  bool stg, hipStream_t st) {
  switch (base) {
    case 5: return k64::launch_sk<256, 256, 4>(g, s, grid, a_t, b_t, stg, st);
    case 6: return k64::launch_sk<256, 128, 4>(g, s, grid, a_t, b_t, stg, st);
    case 7: return k64::launch_sk<128, 128, 2>(g, s, grid, a_t, b_t, stg, st);
    case 8: return k64::launch_sk<128, 256, 4>(g, s, grid, a_t, b_t, stg, st);
    case k64::kT192: return k64::launch_sk<256, 192, 2, 4>(g, s, grid, a_t, b_t, stg, st);
    case k64::kT192S: return k64::launch_sk<128, 192, 2, 2>(g, s, grid, a_t, b_t, stg, st);
    default: return hipErrorInvalidValue;
  }
}
