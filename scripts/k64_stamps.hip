// Diagnostic build of csrc/gemm_k64.hip's two-phase K loop with in-kernel s_memtime stamps
// (cdna_hip_programming.md "In-kernel stamps"): per segment, the share of the loop's cycles,
// averaged over every wave, separately for the two staggered wave groups.  Only SHARES are
// meaningful (the stamps' lgkmcnt(0) fences forbid overlaps the real kernel has).
//
//   hipcc -O3 --offload-arch=gfx950 -DDTA_K64_STAMP -I distributed_training_amd/csrc \
//         scripts/k64_stamps.hip -o /tmp/k64_stamps && /tmp/k64_stamps M N K layout tile
#include "../distributed_training_amd/csrc/gemm_k64.hip"
#include "../distributed_training_amd/csrc/gemm_k64_sk.hip"

#include <cstdio>
#include <vector>

extern unsigned long long* dta_k64_stamp_buf;

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void fill(bf16* p, int64_t n, unsigned seed, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (bf16)(((x & 0xffff) / 32768.f - 1.f) * scale);
  }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 8192, N = argc > 2 ? atoi(argv[2]) : 4096, K = argc > 3 ? atoi(argv[3]) : 4096;
  const char* lay = argc > 4 ? argv[4] : "nt";
  const int tile = argc > 5 ? atoi(argv[5]) : 5;
  const bool at = lay[0] == 't', bt = lay[1] == 'n' && lay[0] != 'n' ? false : (lay[1] == 'n');
  // nt: a [M][K], b [N][K]; nn: b [K][N]; tn: a [K][M], b [K][N]
  const bool b_t = (lay[0] == 'n' && lay[1] == 'n') || (lay[0] == 't');
  (void)bt;
  const int t = dta_gemm_k64_tile(M, N, K, tile);
  if (!t || t <= 4) { fprintf(stderr, "tile %d does not cover / not a two-phase tile\n", tile); return 2; }
  const int bm = k64::tile_bm(t - 4), bn = k64::tile_bn(t - 4), nw = (bm == 128 && bn == 128) ? 4 : 8;
  const int blocks = (M / bm) * (N / bn);
  bf16 *a, *b, *c;
  CK(hipMalloc(&a, (size_t)M * K * 2));
  CK(hipMalloc(&b, (size_t)N * K * 2));
  CK(hipMalloc(&c, (size_t)M * N * 2));
  CK(hipMalloc(&dta_k64_stamp_buf, (size_t)blocks * nw * 10 * 8));
  fill<<<1024, 256>>>(a, (int64_t)M * K, 1u, 1.f);
  fill<<<1024, 256>>>(b, (int64_t)N * K, 2u, 0.02f);
  const int64_t lda = at ? M : K, ldb = b_t ? N : K;
  for (int r = 0; r < 3; ++r)
    CK(dta_gemm_k64(a, lda, at, b, ldb, b_t, c, N, nullptr, 0, nullptr, M, N, K, 1.f, nullptr, 0, nullptr, 0, t, 0));
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> h((size_t)blocks * nw * 10);
  CK(hipMemcpy(h.data(), dta_k64_stamp_buf, h.size() * 8, hipMemcpyDeviceToHost));
  const char* names[10] = {"S1 read+dma issue (+read wait)", "S1 lgkm+vmcnt", "S1 barrier", "S1 32 mfma", "S1 end barrier",
                           "S3 read+dma issue (+read wait)", "S3 lgkm+vmcnt", "S3 barrier", "S3 32 mfma", "S3 end barrier"};
  for (int grp = 0; grp < 2; ++grp) {
    double sum[10] = {0}, tot = 0;
    for (int bl = 0; bl < blocks; ++bl)
      for (int w = 0; w < nw; ++w) {
        if ((w >= nw / 2) != grp) continue;
        for (int i = 0; i < 10; ++i) { sum[i] += h[((size_t)bl * nw + w) * 10 + i]; tot += h[((size_t)bl * nw + w) * 10 + i]; }
      }
    const double per_kt = tot / (blocks * (nw / 2)) / (K / 64);
    printf("%s M %d N %d K %d tile %d  wave group %d: %.0f memtime ticks per K-tile per wave\n", lay, M, N, K, t, grp, per_kt);
    for (int i = 0; i < 10; ++i) printf("  %-34s %5.1f %%\n", names[i], 100.0 * sum[i] / tot);
  }
  return 0;
}
