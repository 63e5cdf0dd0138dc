// Where a k64 GEMM's time goes outside its K loop (verdict r5 item 2: the fixed cost per call): a diagnostic
// build of csrc/gemm_k64.hip with -DDTA_K64_TIMELINE records, per wave, the device real-time clock (100 MHz,
// common to all CUs) at kernel entry, after the K loop's prologue, after the K loop and after the epilogue's
// stores drained, with the wave's CU (HW_ID / XCC_ID).  Per product this prints the kernel span, the mean
// prologue / loop / epilogue of a workgroup per round of tiles, and the hand-over gap on each CU between its
// first workgroup's end and its next workgroup's entry.
//
//   hipcc -O3 --offload-arch=gfx950 -DDTA_K64_TIMELINE -I distributed_training_amd/csrc \
//       scripts/k64_timeline.hip -o runs/bin/k64_timeline && ./runs/bin/k64_timeline
#include "../distributed_training_amd/csrc/gemm_k64.hip"
#include "../distributed_training_amd/csrc/gemm_k64_sk.hip"

// (the W4 tiles live in csrc/gemm_w4.hip, not built here: tile 5 never reaches this)
hipError_t dta_gemm_w4_launch(const k64::Args&, bool, bool, bool, hipStream_t) { return hipErrorNotSupported; }

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

extern unsigned long long* dta_k64_stamp_buf;

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

static int run(int M, int N, int K, bool at, bool bt) {
  const int t = dta_gemm_k64_tile(M, N, K, 5);
  if (t != 5) {
    fprintf(stderr, "tile 5 does not cover %d x %d x %d\n", M, N, K);
    return 2;
  }
  const int NW = 8, blocks = (M / 256) * (N / 256);
  bf16 *a, *b, *c;
  CK(hipMalloc(&a, (size_t)M * K * 2));
  CK(hipMalloc(&b, (size_t)N * K * 2));
  CK(hipMalloc(&c, (size_t)M * N * 2));
  CK(hipMalloc(&dta_k64_stamp_buf, (size_t)blocks * NW * 8 * 8));
  fill<<<1024, 256>>>(a, (int64_t)M * K, 1u, 1.f);
  fill<<<1024, 256>>>(b, (int64_t)N * K, 2u, 0.05f);
  const int64_t lda = at ? M : K, ldb = bt ? N : K;
  auto go = [&]() {
    return dta_gemm_k64(a, lda, at, b, ldb, bt, c, N, nullptr, 0, nullptr, M, N, K, 1.f, nullptr, 0, nullptr, 0, t, 0,
                        nullptr, nullptr, nullptr);
  };
  const char* lay = !at && !bt ? "nt" : (!at ? "nn" : "tn");
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int i = 0; i < 8; ++i) {
    CK(hipEventRecord(e0, 0));
    CK(go());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms * 1e3f);
  }
  std::sort(ts.begin(), ts.end());
  std::vector<unsigned long long> h((size_t)blocks * NW * 8);  // the last launch's stamps
  CK(hipMemcpy(h.data(), dta_k64_stamp_buf, h.size() * 8, hipMemcpyDeviceToHost));
  // per workgroup: wave 0's entry / loop start / loop end / end (the waves of a workgroup are within a barrier)
  struct W { double t0, t1, t2, t3, ti; unsigned long long cu; };
  std::vector<W> w(blocks);
  unsigned long long tmin = ~0ull;
  for (int bl = 0; bl < blocks; ++bl) tmin = std::min(tmin, h[(size_t)bl * NW * 8 + 0]);
  for (int bl = 0; bl < blocks; ++bl) {
    const unsigned long long* s = &h[(size_t)bl * NW * 8];
    const unsigned long long hw = s[4], xcc = s[5];
    // HW_ID: cu_id [11:8], sh_id [12], se_id [15:13]; XCC_ID [3:0]
    const unsigned long long cu = ((xcc & 0xf) << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xf);
    w[bl] = {(s[0] - tmin) * 0.01, (s[1] - tmin) * 0.01, (s[2] - tmin) * 0.01, (s[3] - tmin) * 0.01,
             (s[6] - tmin) * 0.01, cu};
  }
  double span = 0;
  for (auto& x : w) span = std::max(span, x.t3);
  // rounds by entry order on each CU
  std::map<unsigned long long, std::vector<int>> per_cu;
  for (int bl = 0; bl < blocks; ++bl) per_cu[w[bl].cu].push_back(bl);
  const int R = 4;
  double sum[R][7] = {};
  int cnt[R] = {};
  double gap_sum = 0;
  int gap_n = 0;
  for (auto& kv : per_cu) {
    auto& v = kv.second;
    std::sort(v.begin(), v.end(), [&](int x, int y) { return w[x].t0 < w[y].t0; });
    for (size_t i = 0; i < v.size(); ++i) {
      const W& x = w[v[i]];
      const int r = std::min<int>((int)i, R - 1);
      sum[r][0] += x.t0;
      sum[r][1] += x.t1 - x.t0;
      sum[r][2] += x.t2 - x.t1;
      sum[r][3] += x.t3 - x.t2;
      sum[r][4] += x.t3;
      sum[r][5] += x.ti - x.t2;
      cnt[r]++;
      if (i > 0) {
        gap_sum += x.t0 - w[v[i - 1]].t3;
        gap_n++;
      }
    }
  }
  printf("{\"layout\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"tiles\": %d, \"cus_used\": %zu, \"event_us\": %.1f, "
         "\"span_us\": %.1f, \"handover_gap_us\": %.2f, \"rounds\": [",
         lay, M, N, K, blocks, per_cu.size(), ts[ts.size() / 2], span, gap_n ? gap_sum / gap_n : 0.0);
  bool first = true;
  for (int r = 0; r < R; ++r) {
    if (!cnt[r]) continue;
    printf("%s{\"round\": %d, \"workgroups\": %d, \"entry_us\": %.2f, \"prologue_us\": %.2f, \"loop_us\": %.2f, "
           "\"epilogue_us\": %.2f, \"epilogue_issue_us\": %.2f, \"end_us\": %.2f}",
           first ? "" : ", ", r + 1, cnt[r], sum[r][0] / cnt[r], sum[r][1] / cnt[r], sum[r][2] / cnt[r],
           sum[r][3] / cnt[r], sum[r][5] / cnt[r], sum[r][4] / cnt[r]);
    first = false;
  }
  printf("]}\n");
  fflush(stdout);
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(c));
  CK(hipFree(dta_k64_stamp_buf));
  dta_k64_stamp_buf = nullptr;
  return 0;
}

int main(int argc, char** argv) {
  (void)argc;
  (void)argv;
  if (run(8192, 4096, 4096, false, false)) return 1;   // Llama o-proj forward (512 tiles: two rounds)
  if (run(8192, 4096, 14336, false, false)) return 1;  // down-proj forward (same tiles, 3.5x the K loop)
  if (run(8192, 28672, 4096, false, false)) return 1;  // gate/up forward (3584 tiles: 14 rounds)
  if (run(8192, 4096, 4096, false, true)) return 1;    // o-proj input-gradient layout
  return 0;
}
