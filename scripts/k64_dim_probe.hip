// Diagnostic build of csrc/gemm_k64.hip's two-phase loop: with -DDTA_K64_DMA_IN_MFMA=1 each phase's LDS-DMA
// pieces are issued between the MFMAs of its cluster instead of in its read phase.  Times tile id 5
// (256 x 256) on the Llama gate/up (8192 x 28672 x 4096) and o-proj (8192 x 4096 x 4096) products in the
// nt / nn / tn layouts (hipEvent median of 10 after 3 warm-ups), and checks a 1024 x 768 x 1536 product of
// every layout against a naive fp32-accumulate reference kernel.  One JSON line per case.
//
//   hipcc -O3 --offload-arch=gfx950 -DDTA_K64_DMA_IN_MFMA=1 -I distributed_training_amd/csrc \
//       scripts/k64_dim_probe.hip -o runs/bin/k64_dim1 && ./runs/bin/k64_dim1 dim1
#include "../distributed_training_amd/csrc/gemm_k64.hip"
#include "../distributed_training_amd/csrc/gemm_k64_sk.hip"

// (the W4 tiles live in csrc/gemm_w4.hip, not built here: tile 5 never reaches this)
hipError_t dta_gemm_w4_launch(const k64::Args&, bool, bool, bool, hipStream_t) { return hipErrorNotSupported; }

#include <algorithm>
#include <cmath>
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

__global__ void fill(bf16* p, int64_t n, unsigned seed, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (bf16)(((x & 0xffff) / 32768.f - 1.f) * scale);
  }
}

// C[m][n] = sum_k A(m, k) B(n, k); A(m, k) = at ? a[k * M + m] : a[m * K + k]; B(n, k) = bt ? b[k * N + n] : b[n * K + k]
__global__ void ref_gemm(const bf16* a, const bf16* b, float* c, int M, int N, int K, bool at, bool bt) {
  const int m = blockIdx.y, n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k)
    s += (float)(at ? a[(int64_t)k * M + m] : a[(int64_t)m * K + k]) * (float)(bt ? b[(int64_t)k * N + n] : b[(int64_t)n * K + k]);
  c[(int64_t)m * N + n] = s;
}

static int run(const char* tag, int M, int N, int K, bool at, bool bt, bool check) {
  bf16 *a, *b, *c;
  CK(hipMalloc(&a, (size_t)M * K * 2));
  CK(hipMalloc(&b, (size_t)N * K * 2));
  CK(hipMalloc(&c, (size_t)M * N * 2));
  fill<<<1024, 256>>>(a, (int64_t)M * K, 1u, 1.f);
  fill<<<1024, 256>>>(b, (int64_t)N * K, 2u, 0.05f);
  const int64_t lda = at ? M : K, ldb = bt ? N : K;
  const int t = dta_gemm_k64_tile(M, N, K, 5);
  if (t != 5) {
    fprintf(stderr, "tile 5 does not cover %d x %d x %d\n", M, N, K);
    return 2;
  }
  auto go = [&]() {
    return dta_gemm_k64(a, lda, at, b, ldb, bt, c, N, nullptr, 0, nullptr, M, N, K, 1.f, nullptr, 0, nullptr, 0, t, 0,
                        nullptr, nullptr, nullptr);
  };
  const char* lay = !at && !bt ? "nt" : (!at ? "nn" : "tn");
  if (check) {
    CK(go());
    float* r;
    CK(hipMalloc(&r, (size_t)M * N * 4));
    ref_gemm<<<dim3((N + 255) / 256, M), 256>>>(a, b, r, M, N, K, at, bt);
    CK(hipDeviceSynchronize());
    std::vector<float> hr((size_t)M * N);
    std::vector<bf16> hc((size_t)M * N);
    CK(hipMemcpy(hr.data(), r, hr.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hc.data(), c, hc.size() * 2, hipMemcpyDeviceToHost));
    double err = 0, mx = 0;
    for (size_t i = 0; i < hr.size(); ++i) {
      err = std::max(err, (double)std::fabs((float)hc[i] - hr[i]));
      mx = std::max(mx, (double)std::fabs(hr[i]));
    }
    printf("{\"tag\": \"%s\", \"check\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"max_abs_err\": %.5f, \"max_abs_ref\": %.3f, \"ok\": %s}\n",
           tag, lay, M, N, K, err, mx, err <= 8e-3 * mx + 1e-3 ? "true" : "false");
    CK(hipFree(r));
  } else {
    for (int i = 0; i < 3; ++i) CK(go());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int i = 0; i < 10; ++i) {
      CK(hipEventRecord(e0, 0));
      CK(go());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1e3f);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2];
    printf("{\"tag\": \"%s\", \"layout\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"us\": %.1f, \"tflops\": %.1f}\n", tag, lay,
           M, N, K, us, 2.0 * M * N * K / us / 1e6);
  }
  fflush(stdout);
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(c));
  return 0;
}

int main(int argc, char** argv) {
  const char* tag = argc > 1 ? argv[1] : "k64";
  const bool lays[3][2] = {{false, false}, {false, true}, {true, true}};
  for (auto& l : lays)
    if (run(tag, 1024, 768, 1536, l[0], l[1], true)) return 1;
  for (auto& l : lays)
    if (run(tag, 1024, 512, 64, l[0], l[1], true)) return 1;
  const int shapes[4][3] = {{8192, 28672, 4096}, {8192, 4096, 4096}, {8192, 3072, 768}, {8192, 2304, 768}};
  for (auto& s : shapes)
    for (auto& l : lays)
      if (run(tag, s[0], s[1], s[2], l[0], l[1], false)) return 1;
  return 0;
}
