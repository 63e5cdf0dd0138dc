// Diagnostic builds of csrc/optim.hip's flat AdamW (grid cap) timed standalone at the GPT-2 124 M and a
// 1 G parameter size: fp32 master / m / v, bf16 gradients, bf16 copy-out (28 B of HBM traffic per parameter).
// hipEvent medians of 20 launches after 3 warm-ups; prints one JSON line per size.
//
//   hipcc -O3 --offload-arch=gfx950 -DDTA_OPT_MAX_GRID=4096 -I distributed_training_amd/csrc \
//       scripts/adam_diag.hip -o runs/bin/adam_g4096
//   ./runs/bin/adam_g4096 <tag>
#include "../distributed_training_amd/csrc/optim.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const char* tag = argc > 1 ? argv[1] : "adam";
  const int64_t sizes[] = {124475904, 1000000000};
  for (int64_t n : sizes) {
    float *p, *m, *v, *step;
    dta::bf16 *g, *pb;
    CK(hipMalloc(&p, n * 4));
    CK(hipMalloc(&m, n * 4));
    CK(hipMalloc(&v, n * 4));
    CK(hipMalloc(&g, n * 2));
    CK(hipMalloc(&pb, n * 2));
    CK(hipMalloc(&step, 4));
    CK(hipMemset(p, 0, n * 4));
    CK(hipMemset(m, 0, n * 4));
    CK(hipMemset(v, 0, n * 4));
    CK(hipMemset(g, 0, n * 2));
    CK(hipMemset(step, 0, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int i = 0; i < 23; ++i) {
      CK(hipEventRecord(a, 0));
      CK(dta_flat_adam(p, g, 1, m, v, nullptr, pb, n, step, 1e-4f, 0.9f, 0.95f, 1e-8f, 0.1f, 1.f, 1, 0, 0, 1,
                            -1, 0));
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (i >= 3) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float med = ts[ts.size() / 2];
    printf("{\"tag\": \"%s\", \"n\": %lld, \"grid_cap\": %d, \"us\": %.1f, \"TBps\": %.2f}\n", tag, (long long)n,
           DTA_OPT_MAX_GRID, med * 1e3f, 28.0 * n / (med * 1e-3) / 1e12);
    CK(hipFree(p));
    CK(hipFree(m));
    CK(hipFree(v));
    CK(hipFree(g));
    CK(hipFree(pb));
    CK(hipFree(step));
  }
  return 0;
}
