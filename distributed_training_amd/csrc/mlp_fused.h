// Argument block of the fused 2-layer MLP train-step kernel (mlp_fused.hip).
#pragma once
#include <stdint.h>

namespace dta {

enum LossType : int { LOSS_MSE = 0, LOSS_CE = 1 };

struct MlpArgs {
  const float* X;        // [N, in_dim]   device-resident dataset features
  const float* T;        // [N, out_dim]  targets
  const int* idx_ring;   // [ring_steps, idx_stride] sampler indices
  int* cursor;           // global step counter (device)
  unsigned* ticket;      // arrival ticket (zeroed once at setup)
  float* loss_ring;      // [loss_len]
  const float* p_in;     // flat master weights (read)
  float* p_out;          // flat master weights (owner write)
  const float* g_prev;   // previous step's all-reduced gradient (flat)
  float* g_out;          // this step's gradient (flat, pre-scaled)
  const float* mom_in;   // momentum buffers (nullable)
  float* mom_out;
  int64_t o_w1, o_b1, o_w2, o_b2;  // offsets inside the flat buffers (o_w1 == 0, all % 4 == 0)
  int64_t total;                   // flat length (% 4 == 0)
  int in_dim, hidden, out_dim, B;
  int ring_steps, idx_stride, loss_len, own_tiles;
  int act, loss_type, apply_update;
  float grad_scale;
  // SGD hyper-parameters of the pending update
  float lr, momentum, dampening, weight_decay, prev_grad_scale;
  int nesterov, maximize, first_step;
  // diagnostic build only: per-workgroup s_memrealtime stamps at phase ends (nullptr = off)
  unsigned long long* dbg_stamps;
};

}  // namespace dta
