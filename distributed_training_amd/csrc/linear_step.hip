// Fused train step of the reference's default model: ONE nn.Linear(in, out)
// (src/distributed_trainer.py:199, conf/model/default.yaml) with the
// reference's loss (F.cross_entropy against float targets = soft-label CE,
// :163) or MSE, fp32 like the reference, and torch.optim.SGD (:200, :165).
//
// SURVEY.md §2.6 lists ~15 ATen launches per reference step for this model
// (addmm, log_softmax, mul/sum/neg/div, their backwards, mm for dW, sum for
// db, the DDP mul_out/copy kernels, SGD add_).  Here a step is a handful of
// LDS phases inside one workgroup:
//
//   [pending SGD update from the all-reduced gradients of the previous step]
//   gather the batch rows by DistributedSampler index (device index ring)
//   logits z = x W^T + b                    (fp32 FMA, W resident in LDS)
//   loss + dz (soft-label CE or MSE, mean over the batch)
//   dW = dz^T x, db = sum_b dz             (fp32)
//   world size 1: SGD in LDS, next step   |   world size > 1: dW, db * 1/ws -> G_out
//
// Two launch forms share the kernel:
//  * persistent (one rank): `nsteps` complete steps per launch, parameters
//    (and momentum) resident in LDS for the whole launch;
//  * per-step (several ranks): nsteps = 1, the pending update of the previous
//    step is applied first (from the RCCL / p2p all-reduced G_in), this step's
//    gradients go to G_out for the all-reduce that follows in the same graph.
//
// The shapes are tiny (Linear(20, 1): 21 parameters, 32 x 20 batch): this
// is latency-bound VALU work, not MFMA work -- one workgroup, fp32 FMA, no
// global round trips between phases.
#include "common.h"

#include <cstdlib>

namespace dta {

struct LinStepArgs {
  const float* X;         // [N, I] fp32 (device-resident dataset)
  const float* T;         // [N, C] fp32 targets
  const int* ring;        // [R][B] sampler indices
  const int* counts;      // [R] batch size of each slot (last batch of an epoch may be short)
  int* cursor;            // global step counter (slot = cursor % R), advanced by the kernel
  float* P;               // [C*I | C] weight (row-major [C][I]) then bias
  float* M;               // momentum buffer (same layout) or nullptr
  int* flags;             // [0] momentum buffer initialised, [1] G_in holds an update not yet applied
  const float* G_in;      // per-step form: all-reduced gradients of the previous step (or nullptr)
  float* G_out;           // per-step form: this step's gradients * grad_scale (nullptr: persistent form)
  float* loss_ring;       // [loss_len] per-step mean loss
  int* loss_cursor;
  int loss_len;
  int R, B, I, C, nsteps, loss_kind;  // loss_kind: 0 = MSE, 1 = soft-label cross-entropy
  float lr, momentum, dampening, weight_decay, grad_scale;
  int nesterov, maximize;
};

constexpr int kLinThreads = 256;
constexpr int kLinMaxParams = 8192;  // C*I + C fp32 in LDS (x2 with momentum)
constexpr int kLinMaxBI = 8192;      // batch rows in LDS (B*I fp32)
constexpr int kLinMaxBC = 2048;      // B*C logits / targets / dz

__device__ __forceinline__ float sgd_update(float p, float g, float* m, bool started, const LinStepArgs& a) {
  float d = a.maximize ? -g : g;
  if (a.weight_decay != 0.f) d += a.weight_decay * p;
  if (m) {
    const float buf = started ? a.momentum * (*m) + (1.f - a.dampening) * d : d;
    *m = buf;
    d = a.nesterov ? d + a.momentum * buf : buf;
  }
  return p - a.lr * d;
}

// same update, momentum as a (register-resident) reference; `use_m` = momentum buffer present
__device__ __forceinline__ float sgd_update_r(float p, float g, float& m, bool use_m, bool started,
                                              const LinStepArgs& a) {
  float d = a.maximize ? -g : g;
  if (a.weight_decay != 0.f) d += a.weight_decay * p;
  if (use_m) {
    const float buf = started ? a.momentum * m + (1.f - a.dampening) * d : d;
    m = buf;
    d = a.nesterov ? d + a.momentum * buf : buf;
  }
  return p - a.lr * d;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kLinThreads / 64; ++i) s += red[i];
  return s;
}

__global__ void __launch_bounds__(kLinThreads) linear_step_kernel(LinStepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int I = a.I, C = a.C, NP = C * I + C;
  float* p_s = lds;                                  // [NP]
  float* m_s = p_s + NP;                             // [NP] (momentum) -- present only with M
  float* x_s = m_s + (a.M ? NP : 0);                 // [B][I]
  float* t_s = x_s + a.B * I;                        // [B][C]
  float* z_s = t_s + a.B * C;                        // [B][C] logits, then dz
  float* red = z_s + a.B * C;                        // [4] block reduction
  const int tid = threadIdx.x;

  for (int e = tid; e < NP; e += kLinThreads) {
    p_s[e] = a.P[e];
    if (a.M) m_s[e] = a.M[e];
  }
  bool started = a.M ? (a.flags[0] != 0) : false;
  const bool pending = a.G_in != nullptr && a.flags[1] != 0;
  __syncthreads();
  // per-step form: the previous step's update, from the all-reduced gradients
  // (every launch of an epoch is the same graph node; the flag says whether
  // there is an update to apply -- the first step after a flush has none)
  if (pending) {
    for (int e = tid; e < NP; e += kLinThreads) p_s[e] = sgd_update(p_s[e], a.G_in[e], a.M ? &m_s[e] : nullptr, started, a);
    started = true;
    __syncthreads();
  }
  const int cur0 = *a.cursor;
  // Prefetch pipeline (batch rows fit KX / KT registers per thread, e.g. 32 x 20):
  // the next step's sampler indices load while this step's logits are formed and
  // its feature / target rows while this step's loss and gradients are -- the two
  // dependent global round trips of a gather leave the step's critical path.
  constexpr int KX = 4, KT = 1;
  const bool pf = a.B * I <= KX * kLinThreads && a.B * C <= KT * kLinThreads;
  int rx[KX], rt[KT], nb_next = 0;
  float xr[KX], tr[KT];
  auto fetch_idx = [&](int s) {  // sampler rows of step s (ring rows are B wide; unused entries are 0)
    const int slot = (cur0 + s) % a.R;
    const int* idx = a.ring + (int64_t)slot * a.B;
    nb_next = a.counts[slot];
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      const int e = tid + k * kLinThreads;
      rx[k] = e < a.B * I ? idx[e / I] : 0;
    }
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int e = tid + k * kLinThreads;
      rt[k] = e < a.B * C ? idx[e / C] : 0;
    }
  };
  auto fetch_rows = [&]() {
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      const int e = tid + k * kLinThreads;
      if (e < nb_next * I) xr[k] = a.X[(int64_t)rx[k] * I + (e % I)];
    }
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int e = tid + k * kLinThreads;
      if (e < nb_next * C) tr[k] = a.T[(int64_t)rt[k] * C + (e % C)];
    }
  };
  if (pf && a.nsteps > 0) {
    fetch_idx(0);
    fetch_rows();
  }
  for (int s = 0; s < a.nsteps; ++s) {
    const int slot = (cur0 + s) % a.R;
    int nb;
    if (pf) {
      nb = nb_next;
#pragma unroll
      for (int k = 0; k < KX; ++k) {
        const int e = tid + k * kLinThreads;
        if (e < nb * I) x_s[e] = xr[k];
      }
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        const int e = tid + k * kLinThreads;
        if (e < nb * C) t_s[e] = tr[k];
      }
    } else {
      nb = a.counts[slot];
      const int* idx = a.ring + (int64_t)slot * a.B;
      // gather this step's rows (features and targets) into LDS
      for (int e = tid; e < nb * I; e += kLinThreads) {
        const int b = e / I, i = e - b * I;
        x_s[e] = a.X[(int64_t)idx[b] * I + i];
      }
      for (int e = tid; e < nb * C; e += kLinThreads) {
        const int b = e / C, c = e - b * C;
        t_s[e] = a.T[(int64_t)idx[b] * C + c];
      }
    }
    __syncthreads();
    const bool more = pf && s + 1 < a.nsteps;
    if (more) fetch_idx(s + 1);
    // logits
    for (int e = tid; e < nb * C; e += kLinThreads) {
      const int b = e / C, c = e - b * C;
      const float* w = p_s + c * I;
      const float* x = x_s + b * I;
      float z = p_s[C * I + c];
      for (int i = 0; i < I; ++i) z = fmaf(x[i], w[i], z);
      z_s[e] = z;
    }
    __syncthreads();
    if (more) fetch_rows();  // (its indices arrived during the logits)
    // loss and dz (one thread per row)
    float lsum = 0.f;
    for (int b = tid; b < nb; b += kLinThreads) {
      float* z = z_s + b * C;
      const float* t = t_s + b * C;
      if (a.loss_kind == 1) {
        float mx = z[0];
        for (int c = 1; c < C; ++c) mx = fmaxf(mx, z[c]);
        float se = 0.f, ts = 0.f;
        for (int c = 0; c < C; ++c) {
          se += __expf(z[c] - mx);
          ts += t[c];
        }
        const float lse = mx + __logf(se);
        // -sum_c t_c log_softmax(z)_c with log_softmax formed first (as ATen does):
        // one logit gives log_softmax == 0 exactly, hence loss 0
        for (int c = 0; c < C; ++c) lsum -= t[c] * (z[c] - lse);
        const float inv = 1.f / (float)nb;
        for (int c = 0; c < C; ++c) z[c] = (__expf(z[c] - lse) * ts - t[c]) * inv;
      } else {
        const float inv = 2.f / (float)(nb * C);
        for (int c = 0; c < C; ++c) {
          const float d = z[c] - t[c];
          lsum += d * d;
          z[c] = d * inv;
        }
      }
    }
    const float ltot = block_sum(lsum, red);  // (its barriers also publish dz)
    if (tid == 0) {
      const int lc = *a.loss_cursor;
      a.loss_ring[lc % a.loss_len] = a.loss_kind == 1 ? ltot / (float)nb : ltot / (float)(nb * C);
      *a.loss_cursor = lc + 1;
    }
    // gradients; one rank: SGD right here, several ranks: to the exchange buffer
    for (int e = tid; e < NP; e += kLinThreads) {
      float g = 0.f;
      if (e < C * I) {
        const int c = e / I, i = e - c * I;
        for (int b = 0; b < nb; ++b) g = fmaf(z_s[b * C + c], x_s[b * I + i], g);
      } else {
        const int c = e - C * I;
        for (int b = 0; b < nb; ++b) g += z_s[b * C + c];
      }
      if (a.G_out) {
        a.G_out[e] = g * a.grad_scale;
      } else {
        p_s[e] = sgd_update(p_s[e], g, a.M ? &m_s[e] : nullptr, started, a);
      }
    }
    if (!a.G_out) started = true;
    __syncthreads();
  }
  for (int e = tid; e < NP; e += kLinThreads) {
    a.P[e] = p_s[e];
    if (a.M) a.M[e] = m_s[e];
  }
  if (tid == 0) {
    *a.cursor = cur0 + a.nsteps;
    if (a.M && started) a.flags[0] = 1;
    if (a.G_in) a.flags[1] = (a.G_out != nullptr && a.nsteps > 0) ? 1 : 0;  // flush (no G_out): consumed
  }
}

// ------------------------------------------------------------------ one-wave form
// For the reference's own shapes (Linear(20, 1), batch 32) the whole step fits
// ONE wavefront with no LDS and no barrier: lane b owns batch row b (its
// features in registers), every lane holds the (uniform) parameters and
// momenta in registers, the forward is I FMAs per logit, the loss is per lane,
// and each weight / bias gradient is one DPP wave reduction (sum over the
// batch lanes) -- the C*I+C reductions are independent and interleave.  The
// next step's sampler row and feature row are loaded while this step computes
// (two named register sets).  ~20x fewer instructions on the step's critical
// path than the workgroup form above (LDS round trips + 5 barriers).
constexpr int kWI = 32, kWC = 1;  // register-resident limits: in_dim <= 32, out_dim 1, batch <= 64

__global__ void __launch_bounds__(64) linear_step_wave_kernel(LinStepArgs a) {
  const int lane = threadIdx.x;
  const int I = a.I, C = a.C;
  const bool mom = a.M != nullptr;
  float w[kWC][kWI], bb[kWC], mw[kWC][kWI], mb[kWC];
#pragma unroll
  for (int c = 0; c < kWC; ++c) {
#pragma unroll
    for (int i = 0; i < kWI; ++i) {
      const bool live = c < C && i < I;
      w[c][i] = live ? a.P[c * I + i] : 0.f;
      mw[c][i] = live && mom ? a.M[c * I + i] : 0.f;
    }
    bb[c] = c < C ? a.P[C * I + c] : 0.f;
    mb[c] = c < C && mom ? a.M[C * I + c] : 0.f;
  }
  bool started = mom ? (a.flags[0] != 0) : false;
  if (a.G_in != nullptr && a.flags[1] != 0) {  // per-step form: the previous step's all-reduced update
#pragma unroll
    for (int c = 0; c < kWC; ++c) {
      if (c >= C) continue;
#pragma unroll
      for (int i = 0; i < kWI; ++i)
        if (i < I) w[c][i] = sgd_update_r(w[c][i], a.G_in[c * I + i], mw[c][i], mom, started, a);
      bb[c] = sgd_update_r(bb[c], a.G_in[C * I + c], mb[c], mom, started, a);
    }
    started = true;
  }
  const int cur0 = *a.cursor;
  int lc = *a.loss_cursor;
  // three-stage gather pipeline: the sampler row (and batch size) of step s+2 and the
  // feature / target row of step s+1 are in flight while step s computes, so no step
  // waits on a dependent chain of global loads
  auto fetch_idx = [&](int s, int& r, int& nb) {
    const int slot = (cur0 + s) % a.R;
    nb = a.counts[slot];
    r = a.ring[(int64_t)slot * a.B + (lane < a.B ? lane : 0)];
  };
  auto fetch_row = [&](int r, int nb, float (&x)[kWI], float (&t)[kWC]) {
    const bool live = lane < nb;
    const float* row = a.X + (int64_t)(live ? r : 0) * I;  // I % 4 == 0: 16-byte row pieces
#pragma unroll
    for (int j = 0; j < kWI / 4; ++j) {
      const float4 v = (live && 4 * j < I) ? *reinterpret_cast<const float4*>(row + 4 * j)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
      x[4 * j] = v.x;
      x[4 * j + 1] = v.y;
      x[4 * j + 2] = v.z;
      x[4 * j + 3] = v.w;
    }
#pragma unroll
    for (int c = 0; c < kWC; ++c) t[c] = (live && c < C) ? a.T[(int64_t)r * C + c] : 0.f;
  };
  auto step = [&](const float (&x)[kWI], const float (&t)[kWC], int nb) {
    const bool valid = lane < nb;
    float z[kWC], dz[kWC];
#pragma unroll
    for (int c = 0; c < kWC; ++c) {
      z[c] = bb[c];
#pragma unroll
      for (int i = 0; i < kWI; ++i) z[c] = fmaf(x[i], w[c][i], z[c]);
    }
    float lsum = 0.f;
    if (a.loss_kind == 1) {
      float mx = z[0];
#pragma unroll
      for (int c = 1; c < kWC; ++c)
        if (c < C) mx = fmaxf(mx, z[c]);
      float se = 0.f, ts = 0.f;
#pragma unroll
      for (int c = 0; c < kWC; ++c)
        if (c < C) {
          se += __expf(z[c] - mx);
          ts += t[c];
        }
      const float lse = mx + __logf(se);
      const float inv = 1.f / (float)nb;
#pragma unroll
      for (int c = 0; c < kWC; ++c) {
        lsum -= c < C ? t[c] * (z[c] - lse) : 0.f;  // log_softmax first: one logit -> exactly 0
        dz[c] = (valid && c < C) ? (__expf(z[c] - lse) * ts - t[c]) * inv : 0.f;
      }
    } else {
      const float inv = 2.f / (float)(nb * C);
#pragma unroll
      for (int c = 0; c < kWC; ++c) {
        const float d = c < C ? z[c] - t[c] : 0.f;
        lsum += d * d;
        dz[c] = (valid && c < C) ? d * inv : 0.f;
      }
    }
    const float ltot = wave_sum(valid ? lsum : 0.f);
    if (lane == 0) a.loss_ring[lc % a.loss_len] = a.loss_kind == 1 ? ltot / (float)nb : ltot / (float)(nb * C);
    ++lc;
    // gradients: one wave reduction each (uniform result in every lane)
#pragma unroll
    for (int c = 0; c < kWC; ++c) {
      if (c >= C) continue;
#pragma unroll
      for (int i = 0; i < kWI; ++i) {
        if (i >= I) continue;
        const float g = wave_sum(dz[c] * x[i]);
        if (a.G_out) {
          if (lane == 0) a.G_out[c * I + i] = g * a.grad_scale;
        } else {
          w[c][i] = sgd_update_r(w[c][i], g, mw[c][i], mom, started, a);
        }
      }
      const float gb = wave_sum(dz[c]);
      if (a.G_out) {
        if (lane == 0) a.G_out[C * I + c] = gb * a.grad_scale;
      } else {
        bb[c] = sgd_update_r(bb[c], gb, mb[c], mom, started, a);
      }
    }
    if (!a.G_out) started = true;
  };
  float x0[kWI], t0[kWC], x1[kWI], t1[kWC];
  int r1 = 0, nb0 = 0, nb1 = 0, r2 = 0, nb2 = 0;
  if (a.nsteps > 0) {
    int r0;
    fetch_idx(0, r0, nb0);
    fetch_row(r0, nb0, x0, t0);
  }
  if (a.nsteps > 1) fetch_idx(1, r1, nb1);
  for (int s = 0; s < a.nsteps; ++s) {
    if (s + 2 < a.nsteps) fetch_idx(s + 2, r2, nb2);
    if (s + 1 < a.nsteps) fetch_row(r1, nb1, x1, t1);
    step(x0, t0, nb0);
#pragma unroll
    for (int i = 0; i < kWI; ++i) x0[i] = x1[i];
#pragma unroll
    for (int c = 0; c < kWC; ++c) t0[c] = t1[c];
    nb0 = nb1;
    r1 = r2;
    nb1 = nb2;
  }
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < kWC; ++c) {
      if (c >= C) continue;
#pragma unroll
      for (int i = 0; i < kWI; ++i)
        if (i < I) {
          a.P[c * I + i] = w[c][i];
          if (mom) a.M[c * I + i] = mw[c][i];
        }
      a.P[C * I + c] = bb[c];
      if (mom) a.M[C * I + c] = mb[c];
    }
    *a.cursor = cur0 + a.nsteps;
    *a.loss_cursor = lc;
    if (mom && started) a.flags[0] = 1;
    if (a.G_in) a.flags[1] = (a.G_out != nullptr && a.nsteps > 0) ? 1 : 0;
  }
}

}  // namespace dta

using namespace dta;

size_t dta_linear_step_lds_bytes(int I, int C, int B, int momentum) {
  const size_t np = (size_t)C * I + C;
  return 4 * (np * (momentum ? 2 : 1) + (size_t)B * I + 2 * (size_t)B * C + 4);
}

int dta_linear_step_supported(int I, int C, int B, int momentum) {
  const int64_t np = (int64_t)C * I + C;
  return I >= 1 && C >= 1 && B >= 1 && np <= kLinMaxParams && (int64_t)B * I <= kLinMaxBI &&
         (int64_t)B * C <= kLinMaxBC && dta_linear_step_lds_bytes(I, C, B, momentum) <= 160 * 1024;
}

hipError_t dta_linear_step(const LinStepArgs* a, hipStream_t st) {
  if (!dta_linear_step_supported(a->I, a->C, a->B, a->M != nullptr) || a->nsteps < 0 || a->R < 1)
    return hipErrorInvalidValue;
  if (a->I <= kWI && a->I % 4 == 0 && a->C <= kWC && a->B <= 64 &&
      reinterpret_cast<uintptr_t>(a->X) % 16 == 0) {  // the reference's own shapes
    hipLaunchKernelGGL(linear_step_wave_kernel, dim3(1), dim3(64), 0, st, *a);
    return hipGetLastError();
  }
  const size_t lds = dta_linear_step_lds_bytes(a->I, a->C, a->B, a->M != nullptr);
  if (lds > 64 * 1024) {
    static bool raised = false;  // dynamic LDS above 64 KiB must be opted into once
    if (!raised) {
      DTA_HIP_CHECK(hipFuncSetAttribute((const void*)linear_step_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        160 * 1024));
      raised = true;
    }
  }
  hipLaunchKernelGGL(linear_step_kernel, dim3(1), dim3(kLinThreads), lds, st, *a);
  return hipGetLastError();
}
