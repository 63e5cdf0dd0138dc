// Flash attention forward / backward for gfx950 (MI355X), bf16 in, fp32 accumulate.
//
// Needed by the GPT-2 small and Llama-3 8B configurations of BASELINE.json
// (the reference itself has no attention: SURVEY.md §5.7).  Layout: tensors
// are [B, S, heads, D] with an arbitrary row (token) stride, so q/k/v can be
// read straight out of a fused QKV projection buffer and O is written ready for
// the output projection (no transposes).  GQA: q head h uses kv head
// h / (H / Hkv).  Causal or full.
//
// FORWARD (one workgroup = 4 waves = 128 query rows of one (batch, head)):
//   S^T = K . Q^T on v_mfma_f32_32x32x16_bf16 with the KEYS on the accumulator
//   rows and the QUERIES on the lanes, so each lane owns one query row: the
//   online-softmax max / sum are per-lane values (plus one lane^32 exchange),
//   and the rescale of O is a per-lane scalar.  P stays in registers and is the
//   B operand of O^T = V^T . P (cdna_hip_programming.md §3 "accumulator tile as
//   operand"; the permuted key order is matched by reading V^T from LDS).
// BACKWARD (one workgroup = 4 waves = 128 keys of one (batch, kv head)):
//   keys on the lanes; K and V fragments live in registers; per 32-row query
//   block S = Q.K^T and dP = dO.V^T are recomputed, P = exp(S - LSE),
//   dS = P (dP - delta); dV^T += dO^T.P and dK^T += Q^T.dS take P / dS as the
//   B operand straight from the accumulators; dQ += dS.K goes through a
//   wave-private LDS transpose of dS and is accumulated with fp32 atomics.
#include "common.h"

namespace dta {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegBig = -1.0e30f;

struct AttnArgs {
  const bf16* q;
  const bf16* k;
  const bf16* v;
  bf16* o;
  float* lse;           // [B, H, S] natural-log LSE of the scaled scores
  const bf16* dout;
  float* delta;         // [B, H, S]  rowsum(dO * O)
  float* dq_acc;        // [B, S, H, D] fp32 accumulation buffer (zeroed)
  bf16* dk;
  bf16* dv;
  int64_t q_sb, q_ss, k_sb, k_ss, v_sb, v_ss;   // batch / token strides (elements); head stride = D
  int64_t o_sb, o_ss, do_sb, do_ss;
  int64_t dk_sb, dk_ss, dv_sb, dv_ss;
  int B, S, H, Hkv;
  float scale;
};

// ------------------------------------------------------------------ forward
template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256) attn_fwd_kernel(AttnArgs a) {
  constexpr int BN = 64;         // keys per block
  constexpr int KS = D + 8;      // LDS row stride of K tile (bf16)
  constexpr int VTS = BN + 8;    // LDS row stride of V^T tile
  constexpr int NKS = D / 16;    // MFMA k-steps over D
  constexpr int NDT = D / 32;    // 32-wide output tiles over D
  __shared__ __attribute__((aligned(16))) bf16 Ks[BN * KS];
  __shared__ __attribute__((aligned(16))) bf16 Vt[D * VTS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int hk = h / (a.H / a.Hkv);
  const int q0 = blockIdx.x * 128 + wave * 32;
  const int qrow = q0 + r32;  // this lane's query row
  const bf16* qbase = a.q + (int64_t)b * a.q_sb + (int64_t)h * D;
  const bf16* kbase = a.k + (int64_t)b * a.k_sb + (int64_t)hk * D;
  const bf16* vbase = a.v + (int64_t)b * a.v_sb + (int64_t)hk * D;

  // Q fragments (B operand of S^T = K.Q^T): lane (col q, half hh) holds Q[q][16ks + 8hh + j]
  bf16x8 qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (qrow < a.S)
      qf[ks] = *reinterpret_cast<const bf16x8*>(qbase + (int64_t)qrow * a.q_ss + ks * 16 + hh * 8);
    else
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = f2bf(0.f);
  }
  const f32x16 zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x16 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) oacc[dt] = zero16;
  float m = kNegBig, l = 0.f;
  const float c = a.scale * kLog2e;

  const int wg_q_end = min(blockIdx.x * 128 + 128, a.S);
  const int kv_end = CAUSAL ? wg_q_end : a.S;
  for (int k0 = 0; k0 < kv_end; k0 += BN) {
    // ---- stage K [BN][D] and V^T [D][BN] (16-byte global loads) ----
    for (int e = tid; e < BN * (D / 8); e += 256) {
      const int key = e / (D / 8), c8 = (e % (D / 8)) * 8;
      bf16x8 kv, vv;
      if (k0 + key < a.S) {
        kv = *reinterpret_cast<const bf16x8*>(kbase + (int64_t)(k0 + key) * a.k_ss + c8);
        vv = *reinterpret_cast<const bf16x8*>(vbase + (int64_t)(k0 + key) * a.v_ss + c8);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) kv[j] = vv[j] = f2bf(0.f);
      }
      *reinterpret_cast<bf16x8*>(Ks + key * KS + c8) = kv;
#pragma unroll
      for (int j = 0; j < 8; ++j) Vt[(c8 + j) * VTS + key] = vv[j];
    }
    __syncthreads();
    // ---- S^T tiles: rows = keys (k0 + t*32 + row), cols = this wave's queries ----
    f32x16 st[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      st[t] = zero16;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (t * 32 + r32) * KS + ks * 16 + hh * 8);
        st[t] = mfma32x32x16(kf, qf[ks], st[t]);
      }
    }
    // ---- scale, mask, online softmax (per-lane query row) ----
    float mblk = kNegBig;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = k0 + t * 32 + mfma32_row(i, lane);
        float s = st[t][i] * c;
        const bool masked = key >= a.S || (CAUSAL && key > qrow);
        s = masked ? kNegBig : s;
        st[t][i] = s;
        mblk = fmaxf(mblk, s);
      }
    mblk = fmaxf(mblk, __shfl_xor(mblk, 32, kWave));
    const float mnew = fmaxf(m, mblk);
    const float alpha = exp2f(m - mnew);
    float lsum = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = exp2f(st[t][i] - mnew);
        st[t][i] = p;
        lsum += p;
      }
    lsum += __shfl_xor(lsum, 32, kWave);
    l = l * alpha + lsum;
    m = mnew;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
    // ---- O^T += V^T . P ----
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[j] = f2bf(st[t][8 * s + j]);
        const int kb = t * 32 + 16 * s + 4 * hh;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const bf16* vr = Vt + (dt * 32 + r32) * VTS + kb;
          const bf16x4 v0 = *reinterpret_cast<const bf16x4*>(vr);
          const bf16x4 v1 = *reinterpret_cast<const bf16x4*>(vr + 8);
          const bf16x8 vf = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
          oacc[dt] = mfma32x32x16(vf, pb, oacc[dt]);
        }
      }
    __syncthreads();
  }
  // ---- epilogue: O = O^T^T / l ; LSE ----
  if (qrow < a.S) {
    const float inv = 1.f / l;
    bf16* orow = a.o + (int64_t)b * a.o_sb + (int64_t)qrow * a.o_ss + (int64_t)h * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // rows 8g + 4hh + 0..3 are 4 consecutive d
        const bf16x4 ov = {f2bf(oacc[dt][4 * g] * inv), f2bf(oacc[dt][4 * g + 1] * inv),
                           f2bf(oacc[dt][4 * g + 2] * inv), f2bf(oacc[dt][4 * g + 3] * inv)};
        *reinterpret_cast<bf16x4*>(orow + dt * 32 + 8 * g + 4 * hh) = ov;
      }
    if (hh == 0) a.lse[((int64_t)b * a.H + h) * a.S + qrow] = (m + log2f(l)) / kLog2e;
  }
}

// ------------------------------------------------------------------ backward
// delta[b,h,q] = sum_d dO * O   (one wave per query row group)
template <int D>
__global__ void __launch_bounds__(256) attn_bwd_delta_kernel(AttnArgs a) {
  const int tid = threadIdx.x;
  const int64_t row = (int64_t)blockIdx.x * 32 + (tid >> 3);  // 8 threads per (b, q, h) row
  const int64_t total = (int64_t)a.B * a.S * a.H;
  if (row >= total) return;
  const int h = row % a.H;
  const int64_t bq = row / a.H;
  const int q = bq % a.S, b = bq / a.S;
  const bf16* o = a.o + (int64_t)b * a.o_sb + (int64_t)q * a.o_ss + (int64_t)h * D;
  const bf16* d = a.dout + (int64_t)b * a.do_sb + (int64_t)q * a.do_ss + (int64_t)h * D;
  float acc = 0.f;
  for (int c = (tid & 7) * 8; c < D; c += 64) {
    const bf16x8 ov = *reinterpret_cast<const bf16x8*>(o + c);
    const bf16x8 dv = *reinterpret_cast<const bf16x8*>(d + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += bf2f(ov[j]) * bf2f(dv[j]);
  }
#pragma unroll
  for (int off = 4; off > 0; off >>= 1) acc += __shfl_xor(acc, off, kWave);
  if ((tid & 7) == 0) a.delta[((int64_t)b * a.H + h) * a.S + q] = acc;
}

template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256) attn_bwd_kernel(AttnArgs a) {
  constexpr int BM = 32;        // query rows per inner block
  constexpr int RS = D + 8;     // row-major tile stride (bf16)
  constexpr int TS = BM + 8;    // transposed tile stride
  constexpr int NKS = D / 16;
  constexpr int NDT = D / 32;
  __shared__ __attribute__((aligned(16))) bf16 Qs[BM * RS];
  __shared__ __attribute__((aligned(16))) bf16 dOs[BM * RS];
  __shared__ __attribute__((aligned(16))) bf16 Qt[D * TS];
  __shared__ __attribute__((aligned(16))) bf16 dOt[D * TS];
  __shared__ __attribute__((aligned(16))) bf16 Ktw[4 * D * TS];   // per wave: K^T [d][32 keys]
  __shared__ __attribute__((aligned(16))) bf16 dSw[4 * BM * TS];  // per wave: dS [q][32 keys]
  __shared__ float lse2[BM], dlt[BM];
  __shared__ __attribute__((aligned(16))) float dQs[BM * D];  // workgroup-level dQ partial (LDS atomics)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  const int bk = blockIdx.y, b = bk / a.Hkv, hk = bk % a.Hkv;
  const int group = a.H / a.Hkv;
  const int kblk0 = blockIdx.x * 128;
  const int key = kblk0 + wave * 32 + r32;  // this lane's key
  const bf16* kbase = a.k + (int64_t)b * a.k_sb + (int64_t)hk * D;
  const bf16* vbase = a.v + (int64_t)b * a.v_sb + (int64_t)hk * D;
  const float c = a.scale * kLog2e;

  bf16x8 kf[NKS], vf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (key < a.S) {
      kf[ks] = *reinterpret_cast<const bf16x8*>(kbase + (int64_t)key * a.k_ss + ks * 16 + hh * 8);
      vf[ks] = *reinterpret_cast<const bf16x8*>(vbase + (int64_t)key * a.v_ss + ks * 16 + hh * 8);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[ks][j] = vf[ks][j] = f2bf(0.f);
    }
  }
  // wave-private K^T tile for dQ = dS . K  (lane r32 holds key r32: write its d column)
  bf16* Kt = Ktw + wave * D * TS;
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) Kt[(ks * 16 + hh * 8 + j) * TS + r32] = kf[ks][j];
  bf16* dSt = dSw + wave * BM * TS;

  const f32x16 zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x16 dvacc[NDT], dkacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dvacc[dt] = dkacc[dt] = zero16;

  const int qstart = CAUSAL ? (kblk0 / BM) * BM : 0;
  for (int hq = hk * group; hq < (hk + 1) * group; ++hq) {
    const bf16* qbase = a.q + (int64_t)b * a.q_sb + (int64_t)hq * D;
    const bf16* dobase = a.dout + (int64_t)b * a.do_sb + (int64_t)hq * D;
    const float* lse_h = a.lse + ((int64_t)b * a.H + hq) * a.S;
    const float* dl_h = a.delta + ((int64_t)b * a.H + hq) * a.S;
    float* dqb = a.dq_acc + (int64_t)b * a.S * a.H * D + (int64_t)hq * D;
    for (int q0 = qstart; q0 < a.S; q0 += BM) {
      __syncthreads();  // previous block's LDS reads are done
      for (int e = tid; e < BM * (D / 8); e += 256) {
        const int qr = e / (D / 8), c8 = (e % (D / 8)) * 8;
        bf16x8 qv, dv;
        if (q0 + qr < a.S) {
          qv = *reinterpret_cast<const bf16x8*>(qbase + (int64_t)(q0 + qr) * a.q_ss + c8);
          dv = *reinterpret_cast<const bf16x8*>(dobase + (int64_t)(q0 + qr) * a.do_ss + c8);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) qv[j] = dv[j] = f2bf(0.f);
        }
        *reinterpret_cast<bf16x8*>(Qs + qr * RS + c8) = qv;
        *reinterpret_cast<bf16x8*>(dOs + qr * RS + c8) = dv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          Qt[(c8 + j) * TS + qr] = qv[j];
          dOt[(c8 + j) * TS + qr] = dv[j];
        }
      }
      if (tid < BM) {
        const int qr = q0 + tid;
        lse2[tid] = qr < a.S ? lse_h[qr] * kLog2e : 0.f;
        dlt[tid] = qr < a.S ? dl_h[qr] : 0.f;
      }
      for (int e = tid; e < BM * D; e += 256) dQs[e] = 0.f;
      __syncthreads();
      // S = Q.K^T and dP = dO.V^T: rows = queries, cols = this wave's keys
      f32x16 s = zero16, dp = zero16;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(Qs + r32 * RS + ks * 16 + hh * 8);
        const bf16x8 da = *reinterpret_cast<const bf16x8*>(dOs + r32 * RS + ks * 16 + hh * 8);
        s = mfma32x32x16(qa, kf[ks], s);
        dp = mfma32x32x16(da, vf[ks], dp);
      }
      f32x16 p, ds;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qi = mfma32_row(i, lane);
        const int qr = q0 + qi;
        const bool masked = qr >= a.S || key >= a.S || (CAUSAL && key > qr);
        const float pv = masked ? 0.f : exp2f(s[i] * c - lse2[qi]);
        p[i] = pv;
        ds[i] = pv * (dp[i] - dlt[qi]);
      }
      // dV^T += dO^T . P ;  dK^T += Q^T . dS   (P / dS are the B operand as they stand)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 pb, db;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pb[j] = f2bf(p[8 * st + j]);
          db[j] = f2bf(ds[8 * st + j]);
        }
        const int qb = 16 * st + 4 * hh;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const bf16* dr = dOt + (dt * 32 + r32) * TS + qb;
          const bf16* qr = Qt + (dt * 32 + r32) * TS + qb;
          const bf16x4 d0 = *reinterpret_cast<const bf16x4*>(dr);
          const bf16x4 d1 = *reinterpret_cast<const bf16x4*>(dr + 8);
          const bf16x4 q0v = *reinterpret_cast<const bf16x4*>(qr);
          const bf16x4 q1v = *reinterpret_cast<const bf16x4*>(qr + 8);
          const bf16x8 dA = {d0[0], d0[1], d0[2], d0[3], d1[0], d1[1], d1[2], d1[3]};
          const bf16x8 qA = {q0v[0], q0v[1], q0v[2], q0v[3], q1v[0], q1v[1], q1v[2], q1v[3]};
          dvacc[dt] = mfma32x32x16(dA, pb, dvacc[dt]);
          dkacc[dt] = mfma32x32x16(qA, db, dkacc[dt]);
        }
      }
      // dQ[q][d] += dS[q][key] . K[key][d]: dS transposed through the wave's LDS tile
#pragma unroll
      for (int i = 0; i < 16; ++i) dSt[mfma32_row(i, lane) * TS + r32] = f2bf(ds[i]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        f32x16 dq = zero16;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 sa = *reinterpret_cast<const bf16x8*>(dSt + r32 * TS + ks * 16 + hh * 8);
          const bf16x8 kb = *reinterpret_cast<const bf16x8*>(Kt + (dt * 32 + r32) * TS + ks * 16 + hh * 8);
          dq = mfma32x32x16(sa, kb, dq);  // rows q, cols d
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) atomicAdd(&dQs[mfma32_row(i, lane) * D + dt * 32 + r32], dq[i]);
      }
      // one global fp32 atomic per element per workgroup (4 waves reduced in LDS first)
      __syncthreads();
      for (int e = tid; e < BM * D; e += 256) {
        const int qr = q0 + e / D;
        if (qr < a.S) atomicAdd(dqb + (int64_t)qr * a.H * D + (e % D), dQs[e] * a.scale);
      }
    }
  }
  // ---- epilogue: dK = (dK^T)^T * scale, dV = (dV^T)^T ----
  if (key < a.S) {
    bf16* dkr = a.dk + (int64_t)b * a.dk_sb + (int64_t)key * a.dk_ss + (int64_t)hk * D;
    bf16* dvr = a.dv + (int64_t)b * a.dv_sb + (int64_t)key * a.dv_ss + (int64_t)hk * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = dt * 32 + 8 * g + 4 * hh;
        const bf16x4 kv = {f2bf(dkacc[dt][4 * g] * a.scale), f2bf(dkacc[dt][4 * g + 1] * a.scale),
                           f2bf(dkacc[dt][4 * g + 2] * a.scale), f2bf(dkacc[dt][4 * g + 3] * a.scale)};
        const bf16x4 vv = {f2bf(dvacc[dt][4 * g]), f2bf(dvacc[dt][4 * g + 1]), f2bf(dvacc[dt][4 * g + 2]),
                           f2bf(dvacc[dt][4 * g + 3])};
        *reinterpret_cast<bf16x4*>(dkr + d0) = kv;
        *reinterpret_cast<bf16x4*>(dvr + d0) = vv;
      }
  }
}

}  // namespace dta

using namespace dta;

template <int D>
static hipError_t fwd_d(const AttnArgs& a, bool causal, hipStream_t st) {
  dim3 grid((a.S + 127) / 128, a.B * a.H);
  if (causal) hipLaunchKernelGGL((attn_fwd_kernel<D, true>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((attn_fwd_kernel<D, false>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

template <int D>
static hipError_t bwd_d(const AttnArgs& a, bool causal, hipStream_t st) {
  const int64_t rows = (int64_t)a.B * a.S * a.H;
  hipLaunchKernelGGL((attn_bwd_delta_kernel<D>), dim3((unsigned)((rows + 31) / 32)), dim3(256), 0, st, a);
  dim3 grid((a.S + 127) / 128, a.B * a.Hkv);
  if (causal) hipLaunchKernelGGL((attn_bwd_kernel<D, true>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((attn_bwd_kernel<D, false>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t dta_attn_fwd(const AttnArgs* a, int D, bool causal, hipStream_t st) {
  if (D == 64) return fwd_d<64>(*a, causal, st);
  if (D == 128) return fwd_d<128>(*a, causal, st);
  return hipErrorInvalidValue;
}

hipError_t dta_attn_bwd(const AttnArgs* a, int D, bool causal, hipStream_t st) {
  if (D == 64) return bwd_d<64>(*a, causal, st);
  if (D == 128) return bwd_d<128>(*a, causal, st);
  return hipErrorInvalidValue;
}
