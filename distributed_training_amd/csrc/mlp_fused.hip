// Fused 2-layer MLP training step for gfx950 (MI355X).
//
// One launch performs, for one DDP rank and one micro-batch:
//   (0) the PENDING optimizer update of the previous step (SGD with momentum /
//       weight decay / nesterov, exactly torch.optim.SGD semantics), applied to
//       the fp32 master weights with the all-reduced gradient of the previous
//       step  -> "optimizer fused into the next forward";
//   (1) the sampler-indexed gather of the device-resident dataset rows
//       (replaces DataLoader collate + pin_memory + H2D, reference
//       src/distributed_trainer.py:176-182, src/data_utils.py:15-16);
//   (2) Linear(IN,H) on MFMA (v_mfma_f32_32x32x16_bf16, bf16 in / fp32 acc)
//       + bias + activation, Linear(H,OUT) + bias -- computed TRANSPOSED
//       (H^T = W1 . X^T: hidden on the accumulator rows, batch on the lanes) so
//       the activation tile feeds the layer-2 MFMA directly as its B operand;
//   (3) the loss (MSE, or soft-target cross-entropy = the reference's
//       F.cross_entropy(output, float targets), src/distributed_trainer.py:163)
//       and dLoss/dY;
//   (4) the full backward on MFMA: dA^T = W2^T dY^T lands in the same register
//       layout as the kept H^T tile; dH^T and A^T are transposed through a
//       wave-private LDS tile and feed dW1 = dH^T X and dW2^T = A^T dY; db1 comes
//       out of the dW1 MFMA as the extra column of a ones-augmented X (no
//       cross-lane shuffles anywhere in the kernel);
//   (5) gradients written pre-scaled by 1/world_size into the flat DDP grad
//       bucket, ready for one RCCL all-reduce.
//
// Work split: workgroup g OWNS hidden columns [g*own_tiles*32, ...).  Every
// workgroup recomputes the (cheap) full forward so that no cross-workgroup
// exchange is needed for Y; each owner writes only its own slice of updated
// weights / gradients.  Because non-owners read the master weights while owners
// write the updated ones, master / momentum / gradient buffers are ping-ponged
// (p_in != p_out, g_prev != g_out); the host alternates them every step, so an
// even number of steps captured in one hipGraph replays cleanly.
//
// The sampler gather is software-pipelined across steps: one extra "stager"
// workgroup (the last block of the grid) reads the device cursor c, gathers the
// micro-batch of step c+1 (indices from the device index ring) into a staging
// slot and advances the cursor -- it is the ONLY reader/writer of the cursor, so
// no cross-workgroup ticket is needed, and its dependent load chain runs beside
// the compute workgroups instead of on the critical path.  Every workgroup of
// the next step then loads its batch from the staging slot in one round trip,
// in parallel with the parameter loads.  A captured multi-step graph therefore
// walks the index ring without host involvement.
#include "common.h"
#include "mlp_fused.h"

namespace dta {

constexpr int XS = 40;     // bf16 row stride of the X tile (K = 32 + 8 pad)
constexpr int TS = 40;     // bf16 row stride of the wave-private transpose tiles
constexpr int NWAVE = 8;   // 512-thread workgroups
constexpr int NTHR = NWAVE * 64;

__device__ __forceinline__ float sgd_apply(float p, float g, float* mbuf, const MlpArgs& a) {
  g *= a.prev_grad_scale;
  if (a.maximize) g = -g;
  if (a.weight_decay != 0.f) g += a.weight_decay * p;
  if (a.momentum != 0.f) {
    float b = a.first_step ? g : a.momentum * (*mbuf) + (1.f - a.dampening) * g;
    *mbuf = b;
    g = a.nesterov ? g + a.momentum * b : b;
  }
  return p - a.lr * g;
}

// Compile-time activation keeps the kernel branch-free and small (a runtime
// switch unrolled over 16 accumulator registers blew the code past the
// instruction cache: 20k ISA lines -> 3.3k).
template <int ACT>
__device__ __forceinline__ float actf(float x) {
  return act_fwd(ACT, x);
}
template <int ACT>
__device__ __forceinline__ float actd(float x) {
  return act_bwd(ACT, x);
}

__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int RT, int ACT>
__global__ void __launch_bounds__(NTHR) mlp2_fused_step_kernel(MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BP = RT * 32;
  constexpr int BPS = BP + 8;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.hidden, IN = a.in_dim, OUT = a.out_dim, B = a.B;
  const int o_b1 = (int)a.o_b1, o_w2 = (int)a.o_w2, o_b2 = (int)a.o_b2;
  const int r32 = lane & 31, hh = lane >> 5;

  float* Pf = reinterpret_cast<float*>(smem);              // [total] fp32 image of the updated flat params
  bf16* Xs = reinterpret_cast<bf16*>(Pf + a.total);        // [BP][XS]   X (+ ones column at IN)
  bf16* XsT = Xs + BP * XS;                                // [32][BPS]  X^T
  bf16* Tw = XsT + 32 * BPS;                               // [NWAVE][2][32][TS] wave-private transposes
  float* Tg = reinterpret_cast<float*>(Tw + NWAVE * 2 * 32 * TS);  // [BP][8] targets
  float* Ys = Tg + BP * 8;                                 // [BP][8]
  float* dYw = Ys + BP * 8;                                // [NWAVE][BP][8] wave-private dY
  float* Mf = dYw + NWAVE * BP * 8;                        // [total] momentum image (momentum only)

#define DTA_STAMP(k) \
  if (a.dbg_stamps && tid == 0) a.dbg_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();
  DTA_STAMP(0);
  if (a.dbg_stamps && tid == 0) a.dbg_stamps[blockIdx.x * 8 + 5] = __builtin_amdgcn_s_memtime();

  // ---------------- the stager workgroup: batch of the NEXT step ----------------
  if (blockIdx.x == gridDim.x - 1) {
    if (wave != 0) return;
    const int cur = *a.cursor;
    const int* idx = a.idx_ring + (int64_t)((cur + 1) % a.ring_steps) * a.idx_stride;
    unsigned short* xs = a.x_stage + (size_t)(1 - a.parity) * kMlpStageRows * kMlpStageCols;
    float* ts = a.t_stage + (size_t)(1 - a.parity) * kMlpStageRows * 8;
    const int rows = min(a.idx_stride, kMlpStageRows);
    for (int r = lane; r < rows; r += 64) {  // rows past the batch read valid zero-padded ring entries
      const int64_t src = idx[r];
      float x[32];
#pragma unroll
      for (int k = 0; k < 32; ++k) x[k] = k < IN ? a.X[src * IN + k] : 0.f;
      float t[8];
#pragma unroll
      for (int o = 0; o < 8; ++o) t[o] = o < OUT ? a.T[src * OUT + o] : 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f2bf(x[c * 8 + j]);
        *reinterpret_cast<bf16x8*>(xs + r * kMlpStageCols + c * 8) = v;
      }
      *reinterpret_cast<float4*>(ts + r * 8) = make_float4(t[0], t[1], t[2], t[3]);
      *reinterpret_cast<float4*>(ts + r * 8 + 4) = make_float4(t[4], t[5], t[6], t[7]);
    }
    // with gather_self the compute workgroups read the cursor too: the host advances it
    if (!a.gather_self && lane == 0) *a.cursor = cur + 1;
    return;
  }

  const int NT = H >> 5;
  const int ct0 = blockIdx.x * a.own_tiles;
  const int ct1 = min(ct0 + a.own_tiles, NT);
  const int h0 = ct0 * 32, h1 = ct1 * 32;
  const bool stager = blockIdx.x == 0 && wave == NWAVE - 1;  // also computes loss + db2
  const int lcur = stager ? *a.loss_cursor : 0;

  // ---------------- phase 0: loads (params first, then the staged batch) ----------------
  constexpr int U = 8;
  const int n4 = (int)(a.total >> 2);
  const bool has_mom = a.mom_in != nullptr;
  float4 pv[U], gv[U], mv[U];
  auto issue = [&](int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e4 = base + u * NTHR + tid;
      pv[u] = gv[u] = mv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e4 < n4) {
        pv[u] = reinterpret_cast<const float4*>(a.p_in)[e4];
        if (a.apply_update) gv[u] = reinterpret_cast<const float4*>(a.g_prev)[e4];
        if (has_mom) mv[u] = reinterpret_cast<const float4*>(a.mom_in)[e4];
      }
    }
  };
  issue(0);

  // the micro-batch: staged by the previous step (one 16-byte load per thread)
  for (int e = tid; e < BP * 8; e += NTHR) Ys[e] = 0.f;
  if (a.gather_self) {
    const int cur = *a.cursor;
    const int* idx = a.idx_ring + (int64_t)(cur % a.ring_steps) * a.idx_stride;
    for (int e = tid; e < BP * 32; e += NTHR) {
      const int r = e >> 5, k = e & 31;
      float v = 0.f;
      if (r < B) {
        if (k < IN) v = a.X[(int64_t)idx[r] * IN + k];
        else if (k == IN) v = 1.f;  // ones column: dW1's extra output column is db1
      }
      const bf16 bv = f2bf(v);
      Xs[r * XS + k] = bv;
      XsT[k * BPS + r] = bv;
    }
    for (int e = tid; e < BP * 8; e += NTHR) {
      const int r = e >> 3, o = e & 7;
      float v = 0.f;
      if (r < B && o < OUT) v = a.T[(int64_t)idx[r] * OUT + o];
      Tg[e] = v;
    }
  } else {
    const unsigned short* xs = a.x_stage + (size_t)a.parity * kMlpStageRows * kMlpStageCols;
    const float* ts = a.t_stage + (size_t)a.parity * kMlpStageRows * 8;
    for (int e = tid; e < BP * 4; e += NTHR) {  // 8 bf16 per thread
      const int r = e >> 2, c8 = (e & 3) * 8;
      bf16x8 v = *reinterpret_cast<const bf16x8*>(xs + r * kMlpStageCols + c8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = c8 + j;
        if (r >= B || k > IN) v[j] = f2bf(0.f);
        else if (k == IN) v[j] = f2bf(1.f);
      }
      *reinterpret_cast<bf16x8*>(Xs + r * XS + c8) = v;
#pragma unroll
      for (int j = 0; j < 8; ++j) XsT[(c8 + j) * BPS + r] = v[j];
    }
    for (int e = tid; e < BP * 2; e += NTHR) {  // 4 floats per thread
      const int r = e >> 1, c4 = (e & 1) * 4;
      float4 v = *reinterpret_cast<const float4*>(ts + r * 8 + c4);
      if (r >= B) v = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(Tg + r * 8 + c4) = v;
    }
  }

  // pending optimizer update -> LDS image(s).  A lean streaming loop: no
  // per-element region / ownership logic (owners write back from LDS below).
  {
    const bool plain = !has_mom && a.weight_decay == 0.f && !a.maximize;
    const float lr_s = a.lr * a.prev_grad_scale;
#pragma unroll 1
    for (int base = 0; base < n4; base += NTHR * U) {
      if (base > 0) issue(base);
      if (!a.apply_update) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e4 = base + u * NTHR + tid;
          if (e4 < n4) {
            reinterpret_cast<float4*>(Pf)[e4] = pv[u];
            if (has_mom) reinterpret_cast<float4*>(Mf)[e4] = mv[u];
          }
        }
      } else if (plain) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e4 = base + u * NTHR + tid;
          if (e4 < n4) {
            float4 p = pv[u];
            p.x -= lr_s * gv[u].x;
            p.y -= lr_s * gv[u].y;
            p.z -= lr_s * gv[u].z;
            p.w -= lr_s * gv[u].w;
            reinterpret_cast<float4*>(Pf)[e4] = p;
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e4 = base + u * NTHR + tid;
          if (e4 < n4) {
            float4 p = pv[u], m = mv[u];
            p.x = sgd_apply(p.x, gv[u].x, &m.x, a);
            p.y = sgd_apply(p.y, gv[u].y, &m.y, a);
            p.z = sgd_apply(p.z, gv[u].z, &m.z, a);
            p.w = sgd_apply(p.w, gv[u].w, &m.w, a);
            reinterpret_cast<float4*>(Pf)[e4] = p;
            if (has_mom) reinterpret_cast<float4*>(Mf)[e4] = m;
          }
        }
      }
    }
  }
  __syncthreads();
  DTA_STAMP(1);
  // owner write-back of the updated slice (all regions 16-byte aligned: h0 % 32 == 0)
  {
    auto copy_out = [&](int lo, int n) {  // n % 4 == 0
      for (int e4 = tid; e4 < (n >> 2); e4 += NTHR) {
        const int e = lo + 4 * e4;
        *reinterpret_cast<float4*>(a.p_out + e) = *reinterpret_cast<const float4*>(Pf + e);
        if (has_mom) *reinterpret_cast<float4*>(a.mom_out + e) = *reinterpret_cast<const float4*>(Mf + e);
      }
    };
    copy_out(h0 * IN, (h1 - h0) * IN);
    copy_out(o_b1 + h0, h1 - h0);
    for (int o = 0; o < OUT; ++o) copy_out(o_w2 + o * H + h0, h1 - h0);
    if (blockIdx.x == 0 && tid < OUT) {
      a.p_out[o_b2 + tid] = Pf[o_b2 + tid];
      if (has_mom) a.mom_out[o_b2 + tid] = Mf[o_b2 + tid];
    }
  }

  // ---------------- phase 1: forward (transposed) ----------------
  const int nks = (IN + 15) >> 4;  // K = 16 steps over the (zero-padded) input dim
  const bool in4 = (IN & 3) == 0;
  const f32x16 zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  // H^T tile (rows = hidden ct*32.., cols = batch rt*32..) = W1 . X^T + b1
  auto fwd_tile = [&](int rt, int ct) -> f32x16 {
    f32x16 acc = zero16;
    const float* wrow = Pf + (ct * 32 + r32) * IN;
    for (int ks = 0; ks < nks; ++ks) {
      const int k0 = ks * 16 + hh * 8;
      float w[8];
      if (in4) {
        const float4 w0 = *reinterpret_cast<const float4*>(wrow + k0);
        const float4 w1 = *reinterpret_cast<const float4*>(wrow + k0 + 4);
        w[0] = w0.x; w[1] = w0.y; w[2] = w0.z; w[3] = w0.w;
        w[4] = w1.x; w[5] = w1.y; w[6] = w1.z; w[7] = w1.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = wrow[k0 + j];  // stays inside the LDS image; masked below
      }
      bf16x8 av;
#pragma unroll
      for (int j = 0; j < 8; ++j) av[j] = f2bf(k0 + j < IN ? w[j] : 0.f);
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(Xs + (rt * 32 + r32) * XS + k0);
      acc = mfma32x32x16(av, bv, acc);
    }
    const float* b1 = Pf + o_b1 + ct * 32 + 4 * hh;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 bb = *reinterpret_cast<const float4*>(b1 + 8 * q);
      acc[4 * q + 0] += bb.x;
      acc[4 * q + 1] += bb.y;
      acc[4 * q + 2] += bb.z;
      acc[4 * q + 3] += bb.w;
    }
    return acc;
  };
  // Y^T (rows = out, cols = batch) += W2 . act(H^T): the activation tile is the
  // B operand as it stands (k order permuted: element j of lane-half hh is
  // hidden row 16s + 8(j>>2) + 4hh + (j&3) of the tile), W2 read in that order.
  f32x16 yacc[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) yacc[rt] = zero16;
  auto layer2 = [&](int rt, int ct, const f32x16& hp) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 bv, av;
#pragma unroll
      for (int j = 0; j < 8; ++j) bv[j] = f2bf(actf<ACT>(hp[8 * s + j]));
      if (r32 < OUT) {
        const float* w2 = Pf + o_w2 + r32 * H + ct * 32 + 16 * s + 4 * hh;
        const float4 wa = *reinterpret_cast<const float4*>(w2);
        const float4 wb = *reinterpret_cast<const float4*>(w2 + 8);
        av[0] = f2bf(wa.x); av[1] = f2bf(wa.y); av[2] = f2bf(wa.z); av[3] = f2bf(wa.w);
        av[4] = f2bf(wb.x); av[5] = f2bf(wb.y); av[6] = f2bf(wb.z); av[7] = f2bf(wb.w);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) av[j] = f2bf(0.f);
      }
      yacc[rt] = mfma32x32x16(av, bv, yacc[rt]);
    }
  };

  f32x16 keep[RT];
  const int my_ct = ct0 + wave;
  const bool owner_wave = my_ct < ct1;  // own_tiles <= NWAVE: one owned tile per wave
  if (owner_wave) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      keep[rt] = fwd_tile(rt, my_ct);
      layer2(rt, my_ct, keep[rt]);
    }
  }
  // the rest of the (redundant) forward, spread over all waves
  {
    const int nrest = NT - (ct1 - ct0);
#pragma unroll 2
    for (int t = wave; t < nrest; t += NWAVE) {
      const int ct = t < ct0 ? t : t + (ct1 - ct0);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const f32x16 hp = fwd_tile(rt, ct);
        layer2(rt, ct, hp);
      }
    }
  }
  // cross-wave reduction of Y^T: rows o < 8 live in registers 0..3
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = mfma32_row(i, lane);
      if (o < OUT) atomicAdd(&Ys[(rt * 32 + r32) * 8 + o], yacc[rt][i]);
    }
  __syncthreads();
  DTA_STAMP(2);

  // ---------------- phase 2: loss + dY (per wave, no further barrier) ----------------
  float* dYme = dYw + wave * BP * 8;
  float lossr = 0.f;
  if (owner_wave || stager) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int r = rt * 32 + r32;
      float dy[8];
#pragma unroll
      for (int o = 0; o < 8; ++o) dy[o] = 0.f;
      if (r < B && hh == 0) {
        float y[8];
#pragma unroll
        for (int o = 0; o < 8; ++o) y[o] = (o < OUT) ? Ys[r * 8 + o] + Pf[o_b2 + o] : 0.f;
        if (a.loss_type == LOSS_MSE) {
          const float inv = 1.f / (float)(B * OUT);
#pragma unroll
          for (int o = 0; o < 8; ++o)
            if (o < OUT) {
              const float d = y[o] - Tg[r * 8 + o];
              lossr += d * d;
              dy[o] = 2.f * d * inv;
            }
        } else {
          float m = -INFINITY;
#pragma unroll
          for (int o = 0; o < 8; ++o)
            if (o < OUT) m = fmaxf(m, y[o]);
          float sx = 0.f, tsum = 0.f;
#pragma unroll
          for (int o = 0; o < 8; ++o)
            if (o < OUT) {
              sx += __expf(y[o] - m);
              tsum += Tg[r * 8 + o];
            }
          const float lse = m + __logf(sx);
          const float inv = 1.f / (float)B;
#pragma unroll
          for (int o = 0; o < 8; ++o)
            if (o < OUT) {
              const float t = Tg[r * 8 + o];
              lossr -= t * (y[o] - lse);
              dy[o] = (__expf(y[o] - lse) * tsum - t) * inv;
            }
        }
      }
      if (hh == 0) {
#pragma unroll
        for (int o = 0; o < 8; ++o) dYme[r * 8 + o] = dy[o];
      }
    }
    wave_lds_fence();
  }
  DTA_STAMP(3);

  // ---------------- phase 3: backward of the owned hidden tile ----------------
  if (owner_wave) {
    const int hcol = my_ct * 32 + r32;  // lane's hidden index for A-operand rows
    // A operand of dA^T = W2^T . dY^T: row h = hcol, k = o = 8hh + j
    bf16x8 aw2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = 8 * hh + j;
      aw2[j] = f2bf(o < OUT ? Pf[o_w2 + o * H + hcol] : 0.f);
    }
    bf16* At = Tw + (wave * 2 + 0) * 32 * TS;  // A^T tile  [h][b]
    bf16* Dt = Tw + (wave * 2 + 1) * 32 * TS;  // dH^T tile [h][b]
    f32x16 dw1 = zero16, dw2 = zero16;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      bf16x8 bdy;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int o = 8 * hh + j;
        bdy[j] = f2bf(o < 8 ? dYme[(rt * 32 + r32) * 8 + (o & 7)] : 0.f);
      }
      const f32x16 dat = mfma32x32x16(aw2, bdy, zero16);  // rows h, cols b (= kept H^T layout)
      const f32x16 hp = keep[rt];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int hr = mfma32_row(i, lane);
        At[hr * TS + r32] = f2bf(actf<ACT>(hp[i]));
        Dt[hr * TS + r32] = f2bf(dat[i] * actd<ACT>(hp[i]));
      }
      wave_lds_fence();
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int kb = ks * 16 + hh * 8;  // batch index inside this row tile
        const bf16x8 adh = *reinterpret_cast<const bf16x8*>(Dt + r32 * TS + kb);
        const bf16x8 bx = *reinterpret_cast<const bf16x8*>(XsT + r32 * BPS + rt * 32 + kb);
        dw1 = mfma32x32x16(adh, bx, dw1);  // rows h, cols i (col IN = db1)
        const bf16x8 aat = *reinterpret_cast<const bf16x8*>(At + r32 * TS + kb);
        bf16x8 bdy2;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          bdy2[j] = f2bf(r32 < OUT ? dYme[(rt * 32 + kb + j) * 8 + (r32 & 7)] : 0.f);
        dw2 = mfma32x32x16(aat, bdy2, dw2);  // rows h, cols o
      }
      wave_lds_fence();
    }
    const float gs = a.grad_scale;
    // predicates hoisted out of the register loops (one branch per store group)
    if (r32 < IN) {
#pragma unroll
      for (int i = 0; i < 16; ++i) a.g_out[(my_ct * 32 + mfma32_row(i, lane)) * IN + r32] = dw1[i] * gs;
    } else if (r32 == IN) {  // rows 8q + 4hh + 0..3 are contiguous: float4 stores
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(a.g_out + o_b1 + my_ct * 32 + 8 * q + 4 * hh) =
            make_float4(dw1[4 * q] * gs, dw1[4 * q + 1] * gs, dw1[4 * q + 2] * gs, dw1[4 * q + 3] * gs);
    }
    if (r32 < OUT) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(a.g_out + o_w2 + r32 * H + my_ct * 32 + 8 * q + 4 * hh) =
            make_float4(dw2[4 * q] * gs, dw2[4 * q + 1] * gs, dw2[4 * q + 2] * gs, dw2[4 * q + 3] * gs);
    }
  }

  // ------- workgroup 0's last wave: loss and db2 -------
  if (stager) {
    const float lsum = wave_sum(lossr);
    if (lane == 0) {
      const float scale = (a.loss_type == LOSS_MSE) ? 1.f / (float)(B * OUT) : 1.f / (float)B;
      a.loss_ring[lcur % a.loss_len] = lsum * scale;
      *a.loss_cursor = lcur + 1;
    }
    for (int o = 0; o < OUT; ++o) {  // db2[o] = sum_b dY[b][o]
      float v = 0.f;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int r = rt * 32 + r32;
        if (hh == 0 && r < B) v += dYme[r * 8 + o];
      }
      v = wave_sum(v);
      if (lane == 0) a.g_out[o_b2 + o] = v * a.grad_scale;
    }
  }
  DTA_STAMP(4);
  if (a.dbg_stamps && tid == 0) a.dbg_stamps[blockIdx.x * 8 + 6] = __builtin_amdgcn_s_memtime();
#undef DTA_STAMP
}

template <int RT, int ACT>
static hipError_t launch_k(const MlpArgs& a, int grid, size_t lds, hipStream_t st) {
  auto k = mlp2_fused_step_kernel<RT, ACT>;
  static bool attr_set = false;  // one flag per instantiation
  if (!attr_set) {
    DTA_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(NTHR), lds, st, a);
  return hipGetLastError();
}

template <int RT>
static hipError_t launch_act(const MlpArgs& a, int grid, size_t lds, hipStream_t st) {
  switch (a.act) {
    case ACT_RELU: return launch_k<RT, ACT_RELU>(a, grid, lds, st);
    case ACT_GELU_TANH: return launch_k<RT, ACT_GELU_TANH>(a, grid, lds, st);
    case ACT_SILU: return launch_k<RT, ACT_SILU>(a, grid, lds, st);
    default: return launch_k<RT, ACT_NONE>(a, grid, lds, st);
  }
}

}  // namespace dta

using namespace dta;

size_t dta_mlp2_lds_bytes(int64_t total, int bpad, int has_mom) {
  return (size_t)total * 4 * (has_mom ? 2 : 1) + (size_t)bpad * XS * 2 + 32 * (size_t)(bpad + 8) * 2 +
         NWAVE * 2 * 32 * TS * 2 + 2 * (size_t)bpad * 32 + (size_t)NWAVE * bpad * 32;
}

// Returns hipErrorInvalidValue for shapes the fused kernel does not cover;
// the Python layer checks the same limits before calling (ops/mlp_fused.py).
hipError_t dta_mlp2_fused_step(const MlpArgs* args, hipStream_t st) {
  const MlpArgs& a = *args;
  if (a.in_dim < 1 || a.in_dim > 31 || a.out_dim < 1 || a.out_dim > 8 || a.hidden % 32 != 0 || a.B < 1 ||
      a.B > 128 || a.own_tiles < 1 || a.own_tiles > NWAVE || a.ring_steps < 1 || a.loss_len < 1 ||
      a.total % 4 != 0 || a.act < 0 || a.act > 3)
    return hipErrorInvalidValue;
  const int RT = (a.B + 31) / 32;
  const int rt = RT <= 1 ? 1 : (RT <= 2 ? 2 : 4);
  const size_t lds = dta_mlp2_lds_bytes(a.total, rt * 32, a.mom_in != nullptr);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int nt = a.hidden / 32;
  const int grid = (nt + a.own_tiles - 1) / a.own_tiles + 1;  // + the stager workgroup
  if (rt == 1) return launch_act<1>(a, grid, lds, st);
  if (rt == 2) return launch_act<2>(a, grid, lds, st);
  return launch_act<4>(a, grid, lds, st);
}
