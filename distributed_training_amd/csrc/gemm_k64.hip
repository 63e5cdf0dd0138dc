// Host side of the 64-deep-stage bf16 GEMM (the kernels: csrc/gemm_k64_kernels.h): tile choice, argument
// checks, the stream-K plan, launches.  SURVEY.md N07.
#include "gemm_k64_kernels.h"

using namespace dta;

hipError_t dta_gemm_w4_launch(const k64::Args& g, bool a_t, bool b_t, bool staged, hipStream_t st);  // gemm_w4.hip
hipError_t dta_gemm_k64_sk_launch(const k64::Args& g, const k64::SkArgs& s, int grid, int base, bool a_t, bool b_t,
                                  bool stg, hipStream_t st);  // gemm_k64_sk.hip

// 0 if the tile does not cover the problem, else the tile id (1-4, or 5-8 for the same tiles with
// the two-phase K loop).  tile = 0: the fewest rounds of resident workgroups weighted by the tile's
// relative efficiency (bigger tiles reuse more per byte).
int dta_gemm_k64_tile(int M, int N, int K, int tile) {
  // W4: any M, N, K multiples of 8 (clamped DMA rows / chunks, predicated stores, zero-filled K tail)
  if (tile == k64::kW4 || tile == k64::kW4S) return K % 8 == 0 && K > 0 && M % 8 == 0 && N % 8 == 0 ? tile : 0;
  if (K % k64::BK || K < k64::BK) return 0;
  if (tile & (k64::kBufDma | k64::kFlatDma | k64::kNoStg)) {  // the same tile, DMA / epilogue form chosen explicitly
    const int bits = tile & (k64::kBufDma | k64::kFlatDma | k64::kNoStg);
    const int t = dta_gemm_k64_tile(M, N, K, tile & ~bits);
    return t ? (t | bits) : 0;
  }
  auto fits = [&](int t) { return M % k64::tile_bm(t) == 0 && N % k64::tile_bn(t) == 0; };
  if (tile == k64::kT192 || tile == k64::kT192S) return fits(tile) ? tile : 0;
  if (tile & k64::kSK) {  // stream-K: a two-phase tile (optionally with the per-fragment epilogue bit)
    const int base = tile & ~(k64::kSK | k64::kNoStg);
    const int tb = base > k64::kTiles && base <= 2 * k64::kTiles ? base - k64::kTiles : base;
    return k64::sk_base(base) && fits(tb) ? tile : 0;
  }
  if (tile) {
    const int base = tile > k64::kTiles ? tile - k64::kTiles : tile;
    return (tile >= 1 && tile <= 2 * k64::kTiles && fits(base)) ? tile : 0;
  }
  static const double eff[5] = {0, 1.0, 0.88, 0.74, 0.88};
  static const int per_cu[5] = {0, 1, 1, 2, 1};
  int best = 0;
  double best_t = 1e30;
  for (int t = 1; t <= k64::kTiles; ++t) {
    if (!fits(t)) continue;
    const int tiles = (M / k64::tile_bm(t)) * (N / k64::tile_bn(t));
    const int slots = 256 * per_cu[t];
    const int rounds = (tiles + slots - 1) / slots;
    const double tt = rounds * (double)k64::tile_bm(t) * k64::tile_bn(t) * per_cu[t] / eff[t];
    if (tt < best_t * 0.999) {
      best_t = tt;
      best = t;
    }
  }
  // the 8-wave tiles in their two-phase form (measured 3-11 % faster at every GPT-2 / Llama shape)
  return best && best != 3 ? best + k64::kTiles : best;
}

// Stream-K plan of a tile id with the kSK bit: the grid (resident workgroups of the tile on this device, or
// fewer where a run would drop below half a tile's K-tiles) and each workgroup's run of K-tile units; returns
// the tile count (the arrival counters the call needs), 0 if the id is not a stream-K id for the shape;
// ws_floats: the fp32 slab space the launch needs (grid x 2 slabs of BM x BN)
int dta_gemm_k64_sk_plan(int M, int N, int K, int tile, int* grid, int* span, int64_t* ws_floats) {
  if (!(tile & k64::kSK) || !dta_gemm_k64_tile(M, N, K, tile)) return 0;
  const int base = tile & ~(k64::kSK | k64::kNoStg);
  const int tb = base > k64::kTiles && base <= 2 * k64::kTiles ? base - k64::kTiles : base;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    hipDeviceProp_t pr;
    ncu = hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&pr, dev) == hipSuccess ? pr.multiProcessorCount : 256;
  }
  const int tiles = (M / k64::tile_bm(tb)) * (N / k64::tile_bn(tb));
  const int nk = K / k64::BK;
  const int64_t units = (int64_t)tiles * nk;
  const int64_t g0 = (int64_t)ncu * k64::sk_per_cu(base);
  int64_t sp = (units + g0 - 1) / g0;
  sp = std::max<int64_t>(sp, (nk + 1) / 2);  // at most three workgroups share a tile
  *span = (int)sp;
  *grid = (int)((units + sp - 1) / sp);
  if (ws_floats) *ws_floats = (int64_t)*grid * 2 * k64::tile_bm(tb) * k64::tile_bn(tb);
  return tiles;
}

#if defined(DTA_K64_STAMP) || defined(DTA_K64_TIMELINE)
unsigned long long* dta_k64_stamp_buf = nullptr;  // diagnostic build (scripts/k64_stamps.hip)
#endif

// epi: 0 none, 2 GELU (c2 != nullptr: c = pre-activation, c2 = gelu), 16 x gelu'(res), 32 + res,
// 64 SwiGLU backward (res = [a | b] rows, c = [da | db] rows, both 2N wide; no bias / c2 / c32)
hipError_t dta_gemm_k64(const void* a, int64_t lda, bool a_t, const void* b, int64_t ldb, bool b_t, void* c,
                        int64_t ldc, void* c2, int64_t ldc2, float* c32, int M, int N, int K, float alpha,
                        const void* bias, int epi, const void* res, int64_t ldr, int tile, hipStream_t st,
                        const float* alpha_dev, float* sk_ws, int* sk_cnt) {
  int sk_grid = 0, sk_span = 0;
  if (tile & k64::kSK) {
    if (!dta_gemm_k64_sk_plan(M, N, K, tile, &sk_grid, &sk_span, nullptr) || !sk_ws || !sk_cnt ||
        epi == k64::EPI_DSWIGLU)
      return hipErrorInvalidValue;
  }
  tile = dta_gemm_k64_tile(M, N, K, tile);
  if (!tile || (!c && !c32)) return hipErrorInvalidValue;
  if (epi == k64::EPI_DSWIGLU && (bias || c32 || !res || c2)) return hipErrorInvalidValue;
  if (tile == k64::kW4 || tile == k64::kW4S) {
    if (epi == k64::EPI_DSWIGLU) return hipErrorInvalidValue;  // (the 64-deep tiles only)
    // buffer-descriptor DMA with 32-bit offsets: every operand byte within 2 GiB of its base; a transposed
    // operand's extent a multiple of 8 (its DMA chunks are clamped whole)
    const int64_t a_bytes = 2 * (a_t ? (int64_t)(K - 1) * lda + M : (int64_t)(M - 1) * lda + K);
    const int64_t b_bytes = 2 * (b_t ? (int64_t)(K - 1) * ldb + N : (int64_t)(N - 1) * ldb + K);
    if (a_bytes >= 0x7fffffffLL || b_bytes >= 0x7fffffffLL || (a_t && M % 8) || (b_t && N % 8))
      return hipErrorInvalidValue;
    if (c32 && epi != k64::EPI_NONE) return hipErrorInvalidValue;
    k64::Args g{};
    g.a = static_cast<const bf16*>(a);
    g.b = static_cast<const bf16*>(b);
    g.c = static_cast<bf16*>(c);
    g.c2 = static_cast<bf16*>(c2);
    g.c32 = c32;
    g.bias = static_cast<const bf16*>(bias);
    g.res = static_cast<const bf16*>(res);
    g.lda = lda;
    g.ldb = ldb;
    g.ldc = ldc;
    g.ldc2 = ldc2;
    g.ldr = ldr;
    g.M = M;
    g.N = N;
    g.K = K;
    g.alpha = alpha;
    g.alpha_dev = alpha_dev;
    g.epi = epi;
    g.tiles_m = (M + 255) / 256;
    g.tiles_n = (N + 255) / 256;
    return dta_gemm_w4_launch(g, a_t, b_t, tile == k64::kW4S, st);
  }
  bool buf = (tile & k64::kFlatDma) == 0;
  // staged: whole 16-B row chunks of c (and c2, res): 8-element row strides, 16-byte aligned bases
  auto rows16 = [](const void* p, int64_t ld) { return p == nullptr || (ld % 8 == 0 && reinterpret_cast<uintptr_t>(p) % 16 == 0); };
  const bool stg = (tile & k64::kNoStg) == 0 && c32 == nullptr && rows16(c, ldc) && rows16(c2, ldc2) &&
                   ((epi != k64::EPI_DGELU && epi != k64::EPI_RES && epi != k64::EPI_DSWIGLU) || rows16(res, ldr));
  tile &= ~(k64::kBufDma | k64::kFlatDma | k64::kNoStg);
  if (buf) {  // 32-bit offsets: every byte of A and B within 2 GiB of its base (descriptor range)
    const int64_t a_bytes = 2 * (a_t ? (int64_t)(K - 1) * lda + M : (int64_t)(M - 1) * lda + K);
    const int64_t b_bytes = 2 * (b_t ? (int64_t)(K - 1) * ldb + N : (int64_t)(N - 1) * ldb + K);
    buf = a_bytes < 0x7fffffffLL && b_bytes < 0x7fffffffLL;
  }
  if (c32 && epi != k64::EPI_NONE) return hipErrorInvalidValue;
  k64::Args g{};
  g.a = static_cast<const bf16*>(a);
  g.b = static_cast<const bf16*>(b);
  g.c = static_cast<bf16*>(c);
  g.c2 = static_cast<bf16*>(c2);
  g.c32 = c32;
  g.bias = static_cast<const bf16*>(bias);
  g.res = static_cast<const bf16*>(res);
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.ldc2 = ldc2;
  g.ldr = ldr;
  g.M = M;
  g.N = N;
  g.K = K;
  g.alpha = alpha;
  g.alpha_dev = alpha_dev;
  g.epi = epi;
#if defined(DTA_K64_STAMP) || defined(DTA_K64_TIMELINE)
  g.stamps = dta_k64_stamp_buf;
#endif
  if (tile & k64::kSK) {
    if (!buf) return hipErrorInvalidValue;  // (buffer-descriptor DMA only)
    const int base = tile & ~k64::kSK;
    const int tb = base > k64::kTiles && base <= 2 * k64::kTiles ? base - k64::kTiles : base;
    g.tiles_m = M / k64::tile_bm(tb);
    g.tiles_n = N / k64::tile_bn(tb);
    const k64::SkArgs s{sk_ws, sk_cnt, sk_span};
    return dta_gemm_k64_sk_launch(g, s, sk_grid, base, a_t, b_t, stg, st);
  }
  if (tile == k64::kT192 || tile == k64::kT192S) {
    g.tiles_m = M / k64::tile_bm(tile);
    g.tiles_n = N / 192;
    return tile == k64::kT192 ? k64::launch_192<256, 2, 4>(g, a_t, b_t, buf, stg, st)
                              : k64::launch_192<128, 2, 2>(g, a_t, b_t, buf, stg, st);
  }
  // K-loop phases per 64-deep stage: 4, or 2 for the ids past kTiles
  const int ph = tile > k64::kTiles ? 2 : 4;
  if (tile > k64::kTiles) tile -= k64::kTiles;
  g.tiles_m = M / k64::tile_bm(tile);
  g.tiles_n = N / k64::tile_bn(tile);
  switch (tile) {
    case 1: return k64::launch_t<256, 256, 4>(g, a_t, b_t, ph, buf, stg, st);
    case 2: return k64::launch_t<256, 128, 4>(g, a_t, b_t, ph, buf, stg, st);
    case 3: return k64::launch_t<128, 128, 2>(g, a_t, b_t, ph, buf, stg, st);
    default: return k64::launch_t<128, 256, 4>(g, a_t, b_t, ph, buf, stg, st);
  }
}

// n problems dW_i[M_i][N_i] (bf16, row stride ldc_i) = A_i^T B_i, A_i = dy [K_i][M_i] (lda_i), B_i = x [K_i][N_i]
// (ldb_i); db_i (bf16 [M_i] or nullptr) = column sums of A_i.  M_i, N_i multiples of 256, K_i of 64.
int dta_gemm_k64_group_max() { return k64::kGroupMax; }

hipError_t dta_gemm_k64_wgrad_group(int n, const void* const* a, const int64_t* lda, const void* const* b,
                                    const int64_t* ldb, void* const* c, const int64_t* ldc, const int* M, const int* N,
                                    const int* K, void* const* db, hipStream_t st) {
  if (n < 1 || n > k64::kGroupMax) return hipErrorInvalidValue;
  k64::GroupArgs ga{};
  ga.n = n;
  int total = 0;
  bool buf = true;
  for (int i = 0; i < n; ++i) {
    if (M[i] % 256 || N[i] % 256 || K[i] % k64::BK || K[i] < k64::BK) return hipErrorInvalidValue;
    k64::Args& g = ga.p[i];
    g.a = static_cast<const bf16*>(a[i]);
    g.b = static_cast<const bf16*>(b[i]);
    g.c = static_cast<bf16*>(c[i]);
    g.lda = lda[i];
    g.ldb = ldb[i];
    g.ldc = ldc[i];
    g.M = M[i];
    g.N = N[i];
    g.K = K[i];
    g.tiles_m = M[i] / 256;
    g.tiles_n = N[i] / 256;
    g.alpha = 1.f;
    g.epi = k64::EPI_NONE;
    g.db = static_cast<bf16*>(db[i]);
    ga.tile_start[i] = total;
    total += g.tiles_m * g.tiles_n;
    buf = buf && 2 * ((int64_t)(K[i] - 1) * lda[i] + M[i]) < 0x7fffffffLL &&
          2 * ((int64_t)(K[i] - 1) * ldb[i] + N[i]) < 0x7fffffffLL;
  }
  ga.tile_start[n] = total;
  if (buf)
    hipLaunchKernelGGL(k64::gemm_k64_group_kernel<true>, dim3(total), dim3(512), 0, st, ga);
  else
    hipLaunchKernelGGL(k64::gemm_k64_group_kernel<false>, dim3(total), dim3(512), 0, st, ga);
  return hipGetLastError();
}
