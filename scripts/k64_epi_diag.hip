// Diagnostic build of csrc/gemm_k64.hip's 256 x 256 two-phase tile (staged epilogue): where does the
// per-tile fixed cost go?  Built three times (DTA_K64_EPI_DIAG = 0 plain stores, 1 stores skipped,
// 2 non-temporal stores); each binary times, per shape, the one-tile-per-workgroup launch and a
// persistent form (256 workgroups walking the tiles, no overlap between tiles) -- medians of
// interleaved rounds (hipEvent), random operands.
//
//   for d in 0 1 2; do hipcc -O3 --offload-arch=gfx950 -DDTA_K64_EPI_DIAG=$d -I distributed_training_amd/csrc \
//       scripts/k64_epi_diag.hip -o /tmp/k64_epi_$d; done; /tmp/k64_epi_0
#include "../distributed_training_amd/csrc/gemm_k64.hip"
#include "../distributed_training_amd/csrc/gemm_k64_sk.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

// (csrc/gemm_w4.hip is not part of this build)
hipError_t dta_gemm_w4_launch(const k64::Args&, bool, bool, bool, hipStream_t) { return hipErrorInvalidValue; }

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

// persistent: workgroup b takes tiles b, b + G, ... (same XCD remap as the plain launch: G % 8 == 0)
__global__ void __launch_bounds__(512) k64_persist(k64::Args g) {
  const int nt = g.tiles_m * g.tiles_n;
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    k64::k64_body<256, 256, 4, false, false, 2, true, false, true>(g, xcd_remap(t, nt));
    __syncthreads();
  }
}

int main() {
  const int shapes[][3] = {{8192, 4096, 4096}, {8192, 6144, 4096}, {8192, 28672, 4096}, {8192, 4096, 14336},
                           {8192, 3072, 768}, {8192, 128256, 4096}, {16384, 4096, 4096}};
  const int64_t maxA = 16384LL * 14336, maxB = 128256LL * 4096, maxC = 8192LL * 128256;
  bf16 *a, *b, *c;
  CK(hipMalloc(&a, maxA * 2));
  CK(hipMalloc(&b, maxB * 2));
  CK(hipMalloc(&c, maxC * 2));
  fill<<<1024, 256>>>(a, maxA, 1u, 1.f);
  fill<<<1024, 256>>>(b, maxB, 2u, 0.02f);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    k64::Args g{};
    g.a = a; g.b = b; g.c = c; g.lda = K; g.ldb = K; g.ldc = N;
    g.M = M; g.N = N; g.K = K; g.alpha = 1.f; g.epi = 0;
    g.tiles_m = M / 256; g.tiles_n = N / 256;
    const int nt = g.tiles_m * g.tiles_n;
    const int reps = std::max(2, (int)(2e5 / ((double)M * N * K * 2 / 1.3e15 * 1e6)));  // ~0.2 s per round
    std::vector<double> tp, tq;
    for (int round = 0; round < 7; ++round) {
      for (int v = 0; v < 2; ++v) {
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) {
          if (v == 0)
            hipLaunchKernelGGL((k64::gemm_k64_kernel<256, 256, 4, false, false, 2, true, true>), dim3(nt), dim3(512), 0, 0, g);
          else
            hipLaunchKernelGGL(k64_persist, dim3(std::min(nt, 256)), dim3(512), 0, 0, g);
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        (v == 0 ? tp : tq).push_back(ms * 1e3 / reps);
      }
    }
    std::sort(tp.begin(), tp.end());
    std::sort(tq.begin(), tq.end());
    const double fl = 2.0 * M * N * K;
    printf("{\"diag\": %d, \"M\": %d, \"N\": %d, \"K\": %d, \"tiles\": %d, \"plain_us\": %.1f, \"plain_tf\": %.0f, "
           "\"persist_us\": %.1f, \"persist_tf\": %.0f}\n",
           DTA_K64_EPI_DIAG, M, N, K, nt, tp[3], fl / tp[3] * 1e-6, tq[3], fl / tq[3] * 1e-6);
    fflush(stdout);
  }
  return 0;
}
