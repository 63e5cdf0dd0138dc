// Python bindings, second translation unit: the reference-default Linear step
// program and the general bf16 GEMM family (registered into the same _C
// module by dta_register_ext, called from bindings.cpp).
//
// As in bindings.cpp, every entry point checks device / dtype / contiguity /
// shape on the host before enqueueing, so a bad call raises in Python
// instead of faulting the GPU.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <vector>

namespace dta {
struct LinStepArgs {
  const float* X;
  const float* T;
  const int* ring;
  const int* counts;
  int* cursor;
  float* P;
  float* M;
  int* flags;
  const float* G_in;
  float* G_out;
  float* loss_ring;
  int* loss_cursor;
  int loss_len;
  int R, B, I, C, nsteps, loss_kind;
  float lr, momentum, dampening, weight_decay, grad_scale;
  int nesterov, maximize;
};
}  // namespace dta

hipError_t dta_linear_step(const dta::LinStepArgs*, hipStream_t);
int dta_gemm_k64_group_max();
hipError_t dta_gemm_w4_wgrad_group(int, const void* const*, const int64_t*, const void* const*, const int64_t*,
                                   void* const*, const int64_t*, const int*, const int*, const int*, void* const*,
                                   hipStream_t);
hipError_t dta_gemm_k64_wgrad_group(int, const void* const*, const int64_t*, const void* const*, const int64_t*,
                                    void* const*, const int64_t*, const int*, const int*, const int*, void* const*,
                                    hipStream_t);
int dta_gemm_k64_tile(int, int, int, int);
int dta_gemm_k64_sk_plan(int, int, int, int, int*, int*, int64_t*);
hipError_t dta_gemm_k64(const void*, int64_t, bool, const void*, int64_t, bool, void*, int64_t, void*, int64_t, float*,
                        int, int, int, float, const void*, int, const void*, int64_t, int, hipStream_t, const float*, float*, int*);
size_t dta_linear_step_lds_bytes(int, int, int, int);
int dta_linear_step_supported(int, int, int, int);

namespace {

hipStream_t stream_of(int64_t s) {
  if (s == -1) return c10::hip::getCurrentHIPStream().stream();
  return reinterpret_cast<hipStream_t>(s);
}

void ok(hipError_t e, const char* what) { TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e)); }

void gpu_contig(const torch::Tensor& t, const char* name, c10::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == dt, name, " has the wrong dtype");
}

bool has(const c10::optional<torch::Tensor>& t) { return t.has_value() && t->defined(); }

void linear_step(torch::Tensor X, torch::Tensor T, torch::Tensor ring, torch::Tensor counts, torch::Tensor cursor,
                 torch::Tensor P, c10::optional<torch::Tensor> M, torch::Tensor flags,
                 c10::optional<torch::Tensor> G_in, c10::optional<torch::Tensor> G_out, torch::Tensor loss_ring,
                 torch::Tensor loss_cursor, int64_t nsteps, int64_t loss_kind, double lr, double momentum,
                 double dampening, double wd, double grad_scale, bool nesterov, bool maximize, int64_t stream) {
  gpu_contig(X, "X", torch::kFloat32);
  gpu_contig(T, "T", torch::kFloat32);
  gpu_contig(ring, "ring", torch::kInt32);
  gpu_contig(counts, "counts", torch::kInt32);
  gpu_contig(cursor, "cursor", torch::kInt32);
  gpu_contig(P, "P", torch::kFloat32);
  gpu_contig(flags, "flags", torch::kInt32);
  gpu_contig(loss_ring, "loss_ring", torch::kFloat32);
  gpu_contig(loss_cursor, "loss_cursor", torch::kInt32);
  TORCH_CHECK(X.dim() == 2 && T.dim() == 2 && X.size(0) == T.size(0), "X [N, I] and T [N, C]");
  TORCH_CHECK(ring.dim() == 2 && counts.numel() == ring.size(0), "ring [R, B], counts [R]");
  const int I = (int)X.size(1), C = (int)T.size(1), B = (int)ring.size(1);
  const int64_t np = (int64_t)C * I + C;
  TORCH_CHECK(P.numel() == np, "P must hold C*I + C parameters");
  TORCH_CHECK(dta_linear_step_supported(I, C, B, has(M)), "linear_step: shape outside the kernel's limits");
  TORCH_CHECK(nsteps >= 0 && loss_kind >= 0 && loss_kind <= 1, "linear_step: bad nsteps / loss");
  TORCH_CHECK(cursor.numel() >= 1 && flags.numel() >= 2 && loss_cursor.numel() >= 1 && loss_ring.numel() >= 1,
              "linear_step: empty state tensor");
  if (has(M)) {
    gpu_contig(*M, "M", torch::kFloat32);
    TORCH_CHECK(M->numel() == np, "M size");
  }
  if (has(G_in)) {
    gpu_contig(*G_in, "G_in", torch::kFloat32);
    TORCH_CHECK(G_in->numel() == np, "G_in size");
  }
  if (has(G_out)) {
    gpu_contig(*G_out, "G_out", torch::kFloat32);
    TORCH_CHECK(G_out->numel() == np, "G_out size");
  }
  // indices must address rows of X: checked where they are uploaded (host side, FusedLinearProgram)
  dta::LinStepArgs a{};
  a.X = X.data_ptr<float>();
  a.T = T.data_ptr<float>();
  a.ring = ring.data_ptr<int>();
  a.counts = counts.data_ptr<int>();
  a.cursor = cursor.data_ptr<int>();
  a.P = P.data_ptr<float>();
  a.M = has(M) ? M->data_ptr<float>() : nullptr;
  a.flags = flags.data_ptr<int>();
  a.G_in = has(G_in) ? G_in->data_ptr<float>() : nullptr;
  a.G_out = has(G_out) ? G_out->data_ptr<float>() : nullptr;
  a.loss_ring = loss_ring.data_ptr<float>();
  a.loss_cursor = loss_cursor.data_ptr<int>();
  a.loss_len = (int)loss_ring.numel();
  a.R = (int)ring.size(0);
  a.B = B;
  a.I = I;
  a.C = C;
  a.nsteps = (int)nsteps;
  a.loss_kind = (int)loss_kind;
  a.lr = (float)lr;
  a.momentum = (float)momentum;
  a.dampening = (float)dampening;
  a.weight_decay = (float)wd;
  a.grad_scale = (float)grad_scale;
  a.nesterov = nesterov;
  a.maximize = maximize;
  ok(dta_linear_step(&a, stream_of(stream)), "linear_step");
}

bool aligned16(const torch::Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; }

// Grouped weight (+ bias) gradients: dW_i = A_i^T B_i into c_i, db_i = column sums of A_i
// (A_i = dy [K, M_i], B_i = x [K, N_i], c_i [M_i, N_i] bf16; db_i bf16 [M_i] or None).
// impl: 1 = csrc/gemm_k64.hip's grouped kernel (64-deep two-phase loop; M, N multiples of 256, K of 64),
// 2 = csrc/gemm_w4.hip's (4-wave intra-wave interleave; M, N, K multiples of 8; no bias gradients).
void gemm_wgrad_group(std::vector<torch::Tensor> a, std::vector<torch::Tensor> b, std::vector<torch::Tensor> c,
                      std::vector<c10::optional<torch::Tensor>> db, int64_t stream, int64_t impl) {
  const int n = (int)a.size();
  TORCH_CHECK(impl == 1 || impl == 2, "gemm_wgrad_group: impl 1 (k64) or 2 (w4)");
  const bool w4 = impl == 2;
  const int gmax = dta_gemm_k64_group_max();
  TORCH_CHECK(n >= 1 && n <= gmax && (int)b.size() == n && (int)c.size() == n && (int)db.size() == n,
              "gemm_wgrad_group: 1..", gmax, " problems, equal list lengths");
  std::vector<const void*> ap(n), bp(n);
  std::vector<void*> cp(n), dp(n);
  std::vector<int64_t> lda(n), ldb(n), ldc(n);
  std::vector<int> M(n), N(n), K(n);
  for (int i = 0; i < n; ++i) {
    const auto& A = a[i];
    const auto& B = b[i];
    const auto& Cc = c[i];
    for (const auto* t : {&A, &B, &Cc})
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kBFloat16 && t->dim() == 2 && t->stride(1) == 1 &&
                      t->stride(0) % 8 == 0 && aligned16(*t),
                  "gemm_wgrad_group: bf16 2-D GPU tensors, unit inner stride, 16-byte aligned rows");
    TORCH_CHECK(A.size(0) == B.size(0) && Cc.size(0) == A.size(1) && Cc.size(1) == B.size(1),
                "gemm_wgrad_group: A [K, M], B [K, N], C [M, N]");
    if (w4) {
      TORCH_CHECK(A.size(1) % 8 == 0 && B.size(1) % 8 == 0 && A.size(0) % 8 == 0 && A.size(0) > 0 &&
                      A.size(0) < (1 << 30),
                  "gemm_wgrad_group (w4): M, N, K multiples of 8");
    } else {
      TORCH_CHECK(A.size(1) % 256 == 0 && B.size(1) % 256 == 0 && A.size(0) % 64 == 0 && A.size(0) > 0 &&
                      A.size(0) < (1 << 30),
                  "gemm_wgrad_group (k64): M, N multiples of 256, K a multiple of 64");
    }
    ap[i] = A.data_ptr();
    bp[i] = B.data_ptr();
    cp[i] = Cc.data_ptr();
    lda[i] = A.stride(0);
    ldb[i] = B.stride(0);
    ldc[i] = Cc.stride(0);
    M[i] = (int)A.size(1);
    N[i] = (int)B.size(1);
    K[i] = (int)A.size(0);
    dp[i] = nullptr;
    if (db[i] && db[i]->defined()) {
      TORCH_CHECK(!w4, "gemm_wgrad_group (w4): no bias gradients (use the k64 group)");
      const auto& d = *db[i];
      TORCH_CHECK(d.is_cuda() && d.scalar_type() == torch::kBFloat16 && d.is_contiguous() && d.numel() == M[i],
                  "gemm_wgrad_group: db bf16 [M]");
      dp[i] = d.data_ptr();
    }
  }
  ok((w4 ? dta_gemm_w4_wgrad_group : dta_gemm_k64_wgrad_group)(
         n, ap.data(), lda.data(), bp.data(), ldb.data(), cp.data(),
                                                             ldc.data(), M.data(), N.data(), K.data(), dp.data(),
                                                             stream_of(stream)),
     "gemm_wgrad_group");
}

void check_out2d(const torch::Tensor& c, int64_t M, int64_t N, c10::ScalarType dt, const char* what) {
  TORCH_CHECK(c.is_cuda() && c.dim() == 2 && c.size(0) == M && c.size(1) == N && c.stride(1) == 1 &&
                  c.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(c.data_ptr()) % 16 == 0,
              what, ": must be [M, N], unit inner stride, 16-byte aligned rows");
  TORCH_CHECK(c.scalar_type() == dt, what, ": wrong dtype");
}

// The 64-deep-stage GEMM (csrc/gemm_k64.hip).  C[M, N] = alpha * op(A) op(B)^T (+ bias) with epilogue
// epi: 0 none, 2 GELU (out2 given: out = pre-activation h, out2 = gelu(h) -- both returned), 16 x gelu'(res),
// 32 + res.  a: [M, K] (a_t: [K, M]); b: [N, K] (b_t: [K, N]).  alpha_dev: an fp32 device scalar multiplying
// alpha (a loss scale that stays on the GPU).  Returns (out, out2 or None).
std::vector<torch::Tensor> gemm_k64(torch::Tensor a, torch::Tensor b, bool a_t, bool b_t,
                                    c10::optional<torch::Tensor> out, c10::optional<torch::Tensor> out2,
                                    bool out_f32, double alpha, c10::optional<torch::Tensor> bias, int64_t epi,
                                    c10::optional<torch::Tensor> res, int64_t tile, int64_t stream,
                                    c10::optional<torch::Tensor> alpha_dev, c10::optional<torch::Tensor> sk_cnt) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda(), "gemm64: GPU tensors");
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16, "gemm64: bf16 operands");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1, "gemm64: 2-D, unit inner stride");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && aligned16(a) && aligned16(b),
              "gemm64: row strides multiples of 8 elements, 16-byte aligned bases");
  const int64_t M = a_t ? a.size(1) : a.size(0), K = a_t ? a.size(0) : a.size(1);
  const int64_t N = b_t ? b.size(1) : b.size(0), Kb = b_t ? b.size(0) : b.size(1);
  TORCH_CHECK(K == Kb, "gemm64: inner dimensions differ");
  TORCH_CHECK(M < (1 << 30) && N < (1 << 30) && K < (1 << 30), "gemm64: dims too large");
  TORCH_CHECK(dta_gemm_k64_tile((int)M, (int)N, (int)K, (int)tile) != 0,
              "gemm64: shape not covered (M, N multiples of the tile, K a multiple of 64)");
  TORCH_CHECK(epi == 0 || epi == 2 || epi == 16 || epi == 32 || epi == 64,
              "gemm64: epi 0, 2 (gelu), 16 (x gelu'(res)), 32 (+res), 64 (SwiGLU backward)");
  const bool swg = epi == 64;  // res = [a | b] rows and out = [da | db] rows: both [M, 2N]
  TORCH_CHECK(!swg || (!(bias && bias->defined()) && !(out2 && out2->defined())), "gemm64: epi 64 takes no bias / out2");
  TORCH_CHECK(!out_f32 || epi == 0, "gemm64: fp32 output without epilogue only");
  const bool two = out2 && out2->defined();
  TORCH_CHECK(!two || epi == 2, "gemm64: out2 (dual store) with the GELU epilogue only");
  torch::Tensor c, c2;
  if (out && out->defined()) {
    c = *out;
    check_out2d(c, M, swg ? 2 * N : N, out_f32 ? torch::kFloat32 : torch::kBFloat16, "gemm64 out");
  } else {
    c = torch::empty({M, swg ? 2 * N : N}, a.options().dtype(out_f32 ? torch::kFloat32 : torch::kBFloat16));
  }
  if (two) {
    c2 = *out2;
    check_out2d(c2, M, N, torch::kBFloat16, "gemm64 out2");
  }
  const void* bp = nullptr;
  if (bias && bias->defined()) {
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == torch::kBFloat16 && bias->is_contiguous() &&
                    bias->numel() == N && reinterpret_cast<uintptr_t>(bias->data_ptr()) % 8 == 0,
                "gemm64: bias bf16 [N]");
    bp = bias->data_ptr();
  }
  const void* rp = nullptr;
  int64_t ldr = 0;
  TORCH_CHECK((epi == 16 || epi == 32 || swg) == (res && res->defined()), "gemm64: res exactly with epi 16 / 32 / 64");
  if (res && res->defined()) {
    TORCH_CHECK(res->is_cuda() && res->scalar_type() == torch::kBFloat16 && res->dim() == 2 && res->size(0) == M &&
                    res->size(1) == (swg ? 2 * N : N) && res->stride(1) == 1 && res->stride(0) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(res->data_ptr()) % 8 == 0,
                "gemm64: res bf16 [M, N]");
    rp = res->data_ptr();
    ldr = res->stride(0);
  }
  const float* ad = nullptr;
  if (alpha_dev && alpha_dev->defined()) {
    TORCH_CHECK(alpha_dev->is_cuda() && alpha_dev->scalar_type() == torch::kFloat32 && alpha_dev->numel() == 1,
                "gemm64: alpha_dev must be a one-element fp32 GPU tensor");
    ad = alpha_dev->data_ptr<float>();
  }
  // stream-K ids: fp32 slabs for the cut tiles (from the caching allocator, on this stream) and the caller's
  // arrival counters (int32 [>= tiles], zero; the kernel leaves them zero)
  float* skw = nullptr;
  int* skc = nullptr;
  torch::Tensor ws;
  if (tile & 64) {
    int grid = 0, span = 0;
    int64_t wsf = 0;
    const int tiles = dta_gemm_k64_sk_plan((int)M, (int)N, (int)K, (int)tile, &grid, &span, &wsf);
    TORCH_CHECK(tiles > 0, "gemm64: not a stream-K tile for this shape");
    TORCH_CHECK(sk_cnt && sk_cnt->defined() && sk_cnt->is_cuda() && sk_cnt->scalar_type() == torch::kInt32 &&
                    sk_cnt->is_contiguous() && sk_cnt->numel() >= tiles && sk_cnt->device() == a.device(),
                "gemm64: stream-K needs sk_cnt, int32 zeros [>= tiles] on the operands' device");
    ws = torch::empty({wsf}, a.options().dtype(torch::kFloat32));
    skw = ws.data_ptr<float>();
    skc = sk_cnt->data_ptr<int>();
  }
  ok(dta_gemm_k64(a.data_ptr(), a.stride(0), a_t, b.data_ptr(), b.stride(0), b_t, out_f32 ? nullptr : c.data_ptr(),
                  c.stride(0), two ? c2.data_ptr() : nullptr, two ? c2.stride(0) : 0,
                  out_f32 ? c.data_ptr<float>() : nullptr, (int)M, (int)N, (int)K, (float)alpha, bp, (int)epi, rp, ldr,
                  (int)tile, stream_of(stream), ad, skw, skc),
     "gemm64");
  if (two) return {c, c2};
  return {c};
}

}  // namespace

void dta_register_ext(pybind11::module_& m) {
  namespace py = pybind11;
  m.def("linear_step", &linear_step, py::arg("X"), py::arg("T"), py::arg("ring"), py::arg("counts"),
        py::arg("cursor"), py::arg("P"), py::arg("M"), py::arg("flags"), py::arg("G_in"), py::arg("G_out"),
        py::arg("loss_ring"), py::arg("loss_cursor"), py::arg("nsteps"), py::arg("loss_kind"), py::arg("lr"),
        py::arg("momentum"), py::arg("dampening"), py::arg("wd"), py::arg("grad_scale"), py::arg("nesterov"),
        py::arg("maximize"), py::arg("stream") = -1);
  m.def("gemm_wgrad_group", &gemm_wgrad_group, py::arg("a"), py::arg("b"), py::arg("c"), py::arg("db"),
        py::arg("stream") = -1, py::arg("impl") = 1);
  m.def("gemm64_group_max", &dta_gemm_k64_group_max);
  m.def("gemm64", &gemm_k64, py::arg("a"), py::arg("b"), py::arg("a_t") = false, py::arg("b_t") = false,
        py::arg("out") = py::none(), py::arg("out2") = py::none(), py::arg("out_f32") = false, py::arg("alpha") = 1.0,
        py::arg("bias") = py::none(), py::arg("epi") = 0, py::arg("res") = py::none(), py::arg("tile") = 0,
        py::arg("stream") = -1, py::arg("alpha_dev") = py::none(), py::arg("sk_cnt") = py::none());
  m.def("gemm64_sk_plan", [](int M, int N, int K, int tile) {
          int grid = 0, span = 0;
          const int tiles = dta_gemm_k64_sk_plan(M, N, K, tile, &grid, &span, nullptr);
          return std::vector<int>{tiles, grid, span};
        }, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("tile"));
  m.def("gemm64_tile", [](int M, int N, int K, int tile) { return dta_gemm_k64_tile(M, N, K, tile); },
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("tile") = 0);
  m.def("linear_step_supported", [](int I, int C, int B, bool mom) { return dta_linear_step_supported(I, C, B, mom) != 0; });
}
