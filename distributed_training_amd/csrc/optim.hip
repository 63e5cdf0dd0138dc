// Fused optimizer + gradient-bucket kernels for gfx950.
//
// Replaces the per-parameter SGD/AdamW updates and the DDP Reducer's
// "mul_out into bucket / copy_bucket_to_grad" kernels that the reference
// drives through torch (reference call sites
// src/distributed_trainer.py:165 optimizer.step(), ddp_strategy.py:18 DDP).
//
// Design: parameters and gradients live in large flat fp32 buffers owned by
// the DDP/FSDP engines (one contiguous region per bucket / shard), so one
// launch streams an entire bucket with 16-byte vector accesses.  A bf16
// "compute copy" of the parameters can be written in the same pass (fp32
// master -> bf16 copy-out) so no separate cast kernel runs.
#include "common.h"

namespace dta {

struct SgdHyper {
  float lr, momentum, dampening, weight_decay, grad_scale;
  int nesterov, maximize, first_step, vec;
};

__device__ __forceinline__ float sgd_one(float p, float g, float* mbuf, const SgdHyper& h) {
  g *= h.grad_scale;
  if (h.maximize) g = -g;
  if (h.weight_decay != 0.f) g += h.weight_decay * p;
  if (h.momentum != 0.f) {
    float b = h.first_step ? g : h.momentum * (*mbuf) + (1.f - h.dampening) * g;
    *mbuf = b;
    g = h.nesterov ? g + h.momentum * b : b;
  }
  return p - h.lr * g;
}

// p_out may alias p_in (in-place) or be a different buffer (ping-pong).
__global__ void __launch_bounds__(256) flat_sgd_kernel(const float* __restrict__ p_in, float* p_out,
                                                       const float* __restrict__ g, float* mom,
                                                       bf16* __restrict__ p_bf16, int64_t n, SgdHyper h) {
  const int64_t n4 = h.vec ? (n >> 2) : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = reinterpret_cast<const float4*>(p_in)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
    if (mom) m = reinterpret_cast<const float4*>(mom)[i];
    p.x = sgd_one(p.x, gg.x, &m.x, h);
    p.y = sgd_one(p.y, gg.y, &m.y, h);
    p.z = sgd_one(p.z, gg.z, &m.z, h);
    p.w = sgd_one(p.w, gg.w, &m.w, h);
    reinterpret_cast<float4*>(p_out)[i] = p;
    if (mom) reinterpret_cast<float4*>(mom)[i] = m;
    if (p_bf16) {
      bf16x4 o = {f2bf(p.x), f2bf(p.y), f2bf(p.z), f2bf(p.w)};
      reinterpret_cast<bf16x4*>(p_bf16)[i] = o;
    }
  }
  // scalar tail (n % 4)
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float m = mom ? mom[i] : 0.f;
    float p = sgd_one(p_in[i], g[i], &m, h);
    p_out[i] = p;
    if (mom) mom[i] = m;
    if (p_bf16) p_bf16[i] = f2bf(p);
  }
}

struct AdamHyper {
  float lr, beta1, beta2, eps, weight_decay, grad_scale;
  int adamw, maximize, amsgrad, vec;
};

__device__ __forceinline__ float adam_one(float p, float g, float* m, float* v, float* vmax, float bc1,
                                          float bc2_sqrt, const AdamHyper& h) {
  g *= h.grad_scale;
  if (h.maximize) g = -g;
  if (h.weight_decay != 0.f) {
    if (h.adamw) p *= (1.f - h.lr * h.weight_decay);
    else g += h.weight_decay * p;
  }
  float mm = h.beta1 * (*m) + (1.f - h.beta1) * g;
  float vv = h.beta2 * (*v) + (1.f - h.beta2) * g * g;
  *m = mm;
  *v = vv;
  float vuse = vv;
  if (h.amsgrad) {
    vuse = fmaxf(*vmax, vv);
    *vmax = vuse;
  }
  float denom = sqrtf(vuse) / bc2_sqrt + h.eps;
  return p - (h.lr / bc1) * (mm / denom);
}

// `step` is a device counter (float) so the update is hipGraph-replayable:
// the launcher bumps it with a one-thread kernel before this kernel runs.
// Gradients are fp32 or bf16 (the bf16 gradient buffer of a mixed-precision
// flat group is read directly: no fp32 copy of the gradients per step).
__device__ __forceinline__ float4 load_g4(const float* g, int64_t i) { return reinterpret_cast<const float4*>(g)[i]; }
__device__ __forceinline__ float4 load_g4(const bf16* g, int64_t i) {
  const bf16x4 b = reinterpret_cast<const bf16x4*>(g)[i];
  return make_float4(bf2f(b[0]), bf2f(b[1]), bf2f(b[2]), bf2f(b[3]));
}
__device__ __forceinline__ float load_g1(const float* g, int64_t i) { return g[i]; }
__device__ __forceinline__ float load_g1(const bf16* g, int64_t i) { return bf2f(g[i]); }

typedef float nt_f4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld4(const float* a, int64_t i) {
  if constexpr (NT) {
    const nt_f4 v = __builtin_nontemporal_load(reinterpret_cast<const nt_f4*>(a) + i);
    return make_float4(v.x, v.y, v.z, v.w);
  } else {
    return reinterpret_cast<const float4*>(a)[i];
  }
}
template <bool NT>
__device__ __forceinline__ void st4(float* a, int64_t i, const float4 x) {
  if constexpr (NT) __builtin_nontemporal_store(nt_f4{x.x, x.y, x.z, x.w}, reinterpret_cast<nt_f4*>(a) + i);
  else reinterpret_cast<float4*>(a)[i] = x;
}

template <typename GT, bool NT = false>
__global__ void __launch_bounds__(256) flat_adam_kernel(float* __restrict__ p, const GT* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        float* __restrict__ vmax, bf16* __restrict__ p_bf16,
                                                        int64_t n, const float* __restrict__ step,
                                                        AdamHyper h) {
  const float t = *step;
  const float bc1 = 1.f - powf(h.beta1, t);
  const float bc2_sqrt = sqrtf(1.f - powf(h.beta2, t));
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = h.vec ? (n >> 2) : 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = ld4<NT>(p, i);
    float4 gg = load_g4(g, i);
    float4 mm = ld4<NT>(m, i);
    float4 vv = ld4<NT>(v, i);
    float4 xx = make_float4(0.f, 0.f, 0.f, 0.f);
    if (vmax) xx = reinterpret_cast<float4*>(vmax)[i];
    pp.x = adam_one(pp.x, gg.x, &mm.x, &vv.x, &xx.x, bc1, bc2_sqrt, h);
    pp.y = adam_one(pp.y, gg.y, &mm.y, &vv.y, &xx.y, bc1, bc2_sqrt, h);
    pp.z = adam_one(pp.z, gg.z, &mm.z, &vv.z, &xx.z, bc1, bc2_sqrt, h);
    pp.w = adam_one(pp.w, gg.w, &mm.w, &vv.w, &xx.w, bc1, bc2_sqrt, h);
    st4<NT>(p, i, pp);
    st4<NT>(m, i, mm);
    st4<NT>(v, i, vv);
    if (vmax) reinterpret_cast<float4*>(vmax)[i] = xx;
    if (p_bf16) {
      bf16x4 o = {f2bf(pp.x), f2bf(pp.y), f2bf(pp.z), f2bf(pp.w)};
      reinterpret_cast<bf16x4*>(p_bf16)[i] = o;
    }
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float xm = vmax ? vmax[i] : 0.f;
    float mi = m[i], vi = v[i];
    float pi = adam_one(p[i], load_g1(g, i), &mi, &vi, &xm, bc1, bc2_sqrt, h);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if (vmax) vmax[i] = xm;
    if (p_bf16) p_bf16[i] = f2bf(pi);
  }
}

__global__ void step_inc_kernel(float* step) { *step += 1.f; }

// ---------------------------------------------------------------------------
// Multi-tensor apply: up to kMTMaxTensors (src,dst,n) triples and kMTMaxBlocks
// (tensor, chunk) work items per launch, passed by value in the kernarg
// segment (no device metadata allocation -> graph-capturable).
constexpr int kMTMaxTensors = 36;
constexpr int kMTMaxBlocks = 320;
constexpr int kMTChunk = 16384;

struct MTArgs {
  const void* src[kMTMaxTensors];
  void* dst[kMTMaxTensors];
  int64_t n[kMTMaxTensors];
  unsigned char block_tensor[kMTMaxBlocks];
  int block_chunk[kMTMaxBlocks];
};

// dst(float or bf16) = src(float or bf16) * scale ; dtype codes 0=f32 1=bf16
template <typename TS, typename TD>
__global__ void __launch_bounds__(256) mt_scale_copy_kernel(MTArgs a, float scale) {
  const int t = a.block_tensor[blockIdx.x];
  const int64_t c0 = (int64_t)a.block_chunk[blockIdx.x] * kMTChunk;
  const TS* s = reinterpret_cast<const TS*>(a.src[t]);
  TD* d = reinterpret_cast<TD*>(a.dst[t]);
  const int64_t end = min(c0 + (int64_t)kMTChunk, a.n[t]);
  int64_t i0 = c0;
  if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) {
    // 8 elements per thread per iteration (16-byte bf16 / 2x16-byte fp32 accesses)
    const int64_t vend = c0 + (end - c0) / 8 * 8;
    for (int64_t i = c0 + threadIdx.x * 8; i < vend; i += blockDim.x * 8) {
      float v[8];
      load8(s + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= scale;
      store8(d + i, v);
    }
    i0 = vend;
  }
  for (int64_t i = i0 + threadIdx.x; i < end; i += blockDim.x) d[i] = (TD)((float)s[i] * scale);
}

// Sum of squares of a flat buffer -> atomically added into out[0] (fp32).
__global__ void __launch_bounds__(256) flat_sumsq_kernel(const float* __restrict__ x, int64_t n, float* out) {
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = reinterpret_cast<const float4*>(x)[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    acc += x[i] * x[i];
  acc = wave_sum(acc);
  __shared__ float part[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) part[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += part[i];
    atomicAdd(out, s);
  }
}

// x *= min(1, max_norm / (sqrt(sumsq[0]) + 1e-6))   (clip_grad_norm_ semantics)
__global__ void __launch_bounds__(256) flat_clip_kernel(float* __restrict__ x, int64_t n,
                                                        const float* __restrict__ sumsq, float max_norm) {
  const float norm = sqrtf(*sumsq);
  const float coef = fminf(1.f, max_norm / (norm + 1e-6f));
  if (coef >= 1.f) return;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] *= coef;
}

__global__ void __launch_bounds__(256) cast_f32_bf16_kernel(const float* __restrict__ s, bf16* __restrict__ d,
                                                            int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = reinterpret_cast<const float4*>(s)[i];
    bf16x4 o = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
    reinterpret_cast<bf16x4*>(d)[i] = o;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    d[i] = f2bf(s[i]);
}

#ifndef DTA_OPT_MAX_GRID
#define DTA_OPT_MAX_GRID 2048
#endif
static inline int grid_for(int64_t n_vec) {
  int64_t b = (n_vec + 255) / 256;
  if (b > DTA_OPT_MAX_GRID) b = DTA_OPT_MAX_GRID;  // 256 CUs x 8 blocks; grid-stride the rest
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace dta

// ----------------------------- host launchers -----------------------------
using namespace dta;

hipError_t dta_flat_sgd(const float* p_in, float* p_out, const float* g, float* mom, void* p_bf16, int64_t n,
                        float lr, float momentum, float dampening, float wd, float grad_scale, int nesterov,
                        int maximize, int first_step, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  auto al = [](const void* q, int a) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) % a) == 0; };
  const int vec = al(p_in, 16) && al(p_out, 16) && al(g, 16) && al(mom, 16) && al(p_bf16, 8);
  SgdHyper h{lr, momentum, dampening, wd, grad_scale, nesterov, maximize, first_step, vec};
  hipLaunchKernelGGL(flat_sgd_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, st, p_in, p_out, g, mom,
                     reinterpret_cast<bf16*>(p_bf16), n, h);
  return hipGetLastError();
}

hipError_t dta_flat_adam(float* p, const void* g, int g_bf16, float* m, float* v, float* vmax, void* p_bf16,
                         int64_t n, float* step, float lr, float beta1, float beta2, float eps, float wd,
                         float grad_scale, int adamw, int maximize, int amsgrad, int bump_step, int max_blocks,
                         hipStream_t st) {
  if (bump_step) hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step);
  if (n <= 0) return hipGetLastError();
  // max_blocks > 0: a narrow grid (grid-stride) for an update running BESIDE compute-bound kernels on
  // another stream (optimizer inside the backward) -- it then takes a bounded share of the CUs' slots
  const int nb = max_blocks > 0 ? min(grid_for((n + 3) / 4), max_blocks) : grid_for((n + 3) / 4);
  auto al = [](const void* q, int a) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) % a) == 0; };
  const int vec = al(p, 16) && al(g, g_bf16 ? 8 : 16) && al(m, 16) && al(v, 16) && al(vmax, 16) && al(p_bf16, 8);
  AdamHyper h{lr, beta1, beta2, eps, wd, grad_scale, adamw, maximize, amsgrad, vec};
  // bf16 gradients (the mixed-precision engines): the fp32 master / m / v streams non-temporal -- 38.2-38.3 vs
  // 38.9-39.5 ms on Llama-3 8B's 8.03 G parameters, equal at 2 G (scripts/bench_adam.py, profiles/adam_nt_r4.jsonl)
  if (g_bf16)
    hipLaunchKernelGGL((flat_adam_kernel<bf16, true>), dim3(nb), dim3(256), 0, st, p,
                       reinterpret_cast<const bf16*>(g), m, v, vmax, reinterpret_cast<bf16*>(p_bf16), n, step, h);
  else
    hipLaunchKernelGGL(flat_adam_kernel<float>, dim3(nb), dim3(256), 0, st, p,
                       reinterpret_cast<const float*>(g), m, v, vmax, reinterpret_cast<bf16*>(p_bf16), n, step, h);
  return hipGetLastError();
}

hipError_t dta_step_inc(float* step, hipStream_t st) {
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step);
  return hipGetLastError();
}

// Multi-tensor scale-copy over lists.  dtype codes: 0 = f32, 1 = bf16.
hipError_t dta_mt_scale_copy(const void* const* src, void* const* dst, const int64_t* n, int count, int sdt, int ddt,
                             float scale, hipStream_t st) {
  int i = 0;
  int64_t resume_chunk = 0;
  while (i < count) {
    MTArgs a;
    int nt = 0, nb = 0;
    while (i < count && nt < kMTMaxTensors && nb < kMTMaxBlocks) {
      a.src[nt] = src[i];
      a.dst[nt] = dst[i];
      a.n[nt] = n[i];
      const int64_t chunks = (n[i] + kMTChunk - 1) / kMTChunk;
      int64_t c = resume_chunk;
      for (; c < chunks && nb < kMTMaxBlocks; ++c) {
        a.block_tensor[nb] = (unsigned char)nt;
        a.block_chunk[nb] = (int)c;
        ++nb;
      }
      ++nt;
      if (c < chunks) {  // block table full mid-tensor: resume this tensor next launch
        resume_chunk = c;
        break;
      }
      resume_chunk = 0;
      ++i;
    }
    if (nb > 0) {
      if (sdt == 0 && ddt == 0)
        hipLaunchKernelGGL((mt_scale_copy_kernel<float, float>), dim3(nb), dim3(256), 0, st, a, scale);
      else if (sdt == 0 && ddt == 1)
        hipLaunchKernelGGL((mt_scale_copy_kernel<float, bf16>), dim3(nb), dim3(256), 0, st, a, scale);
      else if (sdt == 1 && ddt == 0)
        hipLaunchKernelGGL((mt_scale_copy_kernel<bf16, float>), dim3(nb), dim3(256), 0, st, a, scale);
      else
        hipLaunchKernelGGL((mt_scale_copy_kernel<bf16, bf16>), dim3(nb), dim3(256), 0, st, a, scale);
      DTA_HIP_CHECK(hipGetLastError());
    }
  }
  return hipSuccess;
}

hipError_t dta_flat_sumsq(const float* x, int64_t n, float* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(flat_sumsq_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, st, x, n, out);
  return hipGetLastError();
}

hipError_t dta_flat_clip(float* x, int64_t n, const float* sumsq, float max_norm, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(flat_clip_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, n, sumsq, max_norm);
  return hipGetLastError();
}

hipError_t dta_cast_f32_bf16(const float* s, void* d, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, st, s,
                     reinterpret_cast<bf16*>(d), n);
  return hipGetLastError();
}
