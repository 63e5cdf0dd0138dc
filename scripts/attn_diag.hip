// Diagnostic builds of csrc/attention.hip (prefetch depths, op order) timed standalone on the Llama-3 8B
// (B 1, S 8192, H 32 / Hkv 8, D 128) and GPT-2 (B 8, S 1024, H 12, D 64) causal shapes: forward, and the
// backward's dQ and dK/dV kernels separately (hipEvent medians of interleaved rounds, random operands).
//
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize -DDTA_DKDV_PF=3 \
//       -I distributed_training_amd/csrc scripts/attn_diag.hip -o scripts/attn_diag_pf3
//   DTA_ATTN_BWD_ILV=0|1 ./scripts/attn_diag_pf3 <tag>
#include "../distributed_training_amd/csrc/attention.hip"

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

__global__ void fillr(bf16* p, int64_t n, unsigned seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    // ~N(0, 1)-ish: sum of two uniforms
    const float u = ((x & 0xffff) / 65536.f) + ((x >> 16) / 65536.f) - 1.f;
    p[i] = (bf16)(u * 2.45f);
  }
}

int main(int argc, char** argv) {
  const char* tag = argc > 1 ? argv[1] : "";
  struct Shape { const char* name; int B, S, H, Hkv, D; };
  const Shape shapes[] = {{"llama8b", 1, 8192, 32, 8, 128}, {"gpt2", 8, 1024, 12, 12, 64}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& sh : shapes) {
    const int64_t nq = (int64_t)sh.B * sh.S * sh.H * sh.D, nk = (int64_t)sh.B * sh.S * sh.Hkv * sh.D;
    bf16 *q, *k, *v, *o, *dout, *dq, *dk, *dv;
    float *lse, *delta;
    CK(hipMalloc(&q, nq * 2)); CK(hipMalloc(&o, nq * 2)); CK(hipMalloc(&dout, nq * 2)); CK(hipMalloc(&dq, nq * 2));
    CK(hipMalloc(&k, nk * 2)); CK(hipMalloc(&v, nk * 2)); CK(hipMalloc(&dk, nk * 2)); CK(hipMalloc(&dv, nk * 2));
    CK(hipMalloc(&lse, (int64_t)sh.B * sh.H * sh.S * 4)); CK(hipMalloc(&delta, (int64_t)sh.B * sh.H * sh.S * 4));
    fillr<<<1024, 256>>>(q, nq, 1u); fillr<<<1024, 256>>>(k, nk, 2u); fillr<<<1024, 256>>>(v, nk, 3u);
    fillr<<<1024, 256>>>(dout, nq, 4u);
    AttnArgs a{};
    a.q = q; a.k = k; a.v = v; a.o = o; a.lse = lse; a.dout = dout; a.delta = delta; a.dq = dq; a.dk = dk; a.dv = dv;
    a.q_sb = (int64_t)sh.S * sh.H * sh.D; a.q_ss = sh.H * sh.D; a.o_sb = a.q_sb; a.o_ss = a.q_ss;
    a.do_sb = a.q_sb; a.do_ss = a.q_ss; a.dq_sb = a.q_sb; a.dq_ss = a.q_ss;
    a.k_sb = (int64_t)sh.S * sh.Hkv * sh.D; a.k_ss = sh.Hkv * sh.D; a.v_sb = a.k_sb; a.v_ss = a.k_ss;
    a.dk_sb = a.k_sb; a.dk_ss = a.k_ss; a.dv_sb = a.k_sb; a.dv_ss = a.k_ss;
    a.B = sh.B; a.S = sh.S; a.H = sh.H; a.Hkv = sh.Hkv; a.scale = 1.f / sqrtf((float)sh.D);
    CK(dta_attn_fwd(&a, sh.D, true, 0));
    CK(hipDeviceSynchronize());
    const int reps = sh.D == 128 ? 5 : 50;
    std::vector<double> tf, tb;
    for (int round = 0; round < 7; ++round) {
      for (int which = 0; which < 2; ++which) {
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) CK(which == 0 ? dta_attn_fwd(&a, sh.D, true, 0) : dta_attn_bwd(&a, sh.D, true, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        (which == 0 ? tf : tb).push_back(ms * 1e3 / reps);
      }
    }
    std::sort(tf.begin(), tf.end());
    std::sort(tb.begin(), tb.end());
    const double fl = 2.0 * sh.B * sh.H * (double)sh.S * sh.S * sh.D;
    printf("{\"tag\": \"%s\", \"shape\": \"%s\", \"dkdv_pf\": %d, \"rescale_branch\": %d, \"fwd_us\": %.1f, \"bwd_us\": %.1f, \"fwd_tf\": %.0f, "
           "\"bwd_tf\": %.0f}\n", tag, sh.name, DTA_DKDV_PF, DTA_FWD_RESCALE_BRANCH, tf[3], tb[3], fl / tf[3] * 1e-6, 2.5 * fl / tb[3] * 1e-6);
    fflush(stdout);
    hipFree(q); hipFree(k); hipFree(v); hipFree(o); hipFree(dout); hipFree(dq); hipFree(dk); hipFree(dv);
    hipFree(lse); hipFree(delta);
  }
  return 0;
}
