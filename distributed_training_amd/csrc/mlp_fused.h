// Argument block of the fused 2-layer MLP train-step kernel (mlp_fused.hip).
#pragma once
#include <stdint.h>

namespace dta {

enum LossType : int { LOSS_MSE = 0, LOSS_CE = 1 };

constexpr int kMlpStageRows = 128;  // max micro-batch rows of the staged gather
constexpr int kMlpStageCols = 32;   // bf16 columns per staged row (in_dim <= 31, zero padded)

struct MlpArgs {
  const float* X;        // [N, in_dim]   device-resident dataset features
  const float* T;        // [N, out_dim]  targets
  const int* idx_ring;   // [ring_steps, idx_stride] sampler indices
  int* cursor;           // sampler step counter (device; read/advanced only by the stager workgroup)
  int* loss_cursor;      // loss-ring position (device; read/advanced only by workgroup 0)
  unsigned short* x_stage;  // [2][kMlpStageRows][kMlpStageCols] bf16 bits: gathered batch
  float* t_stage;        // [2][kMlpStageRows][8]
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
  int parity;       // staged batch of THIS step is slot `parity`; next step's goes to 1-parity
  int gather_self;  // 1: gather this step's batch from the ring (first step); cursor not advanced
  float grad_scale;
  // SGD hyper-parameters of the pending update
  float lr, momentum, dampening, weight_decay, prev_grad_scale;
  int nesterov, maximize, first_step;
  // diagnostic build only: per-workgroup s_memrealtime stamps at phase ends (nullptr = off)
  unsigned long long* dbg_stamps;
};

// Persistent single-workgroup train loop (csrc/mlp_persistent.hip)
struct MlpPArgs {
  const void* Xp;        // [Ntot][32] bf16: features, 1.0 at column in, zeros after (prepared once)
  const float* T;        // [Ntot][out]
  const int* idx_ring;   // [ring_steps][idx_stride]
  int* cursor;           // ring row of the next step (advanced by nsteps)
  float* loss_ring;      // mean loss per step
  int* loss_cursor;
  int* mom_started;      // 0 until the first momentum update
  float* P;              // flat fp32 params (in/out)
  float* M;              // flat fp32 momentum (in/out) or null
  int o_w1, o_b1, o_w2, o_b2, total;
  int in_dim, hidden, out_dim, B;
  int ring_steps, idx_stride, loss_len, nsteps;
  int loss_type;
  float grad_scale, lr, momentum, dampening, weight_decay;
  int nesterov, maximize;
  unsigned long long* dbg;  // diagnostic s_memtime stamps [waves][8] of one step (nullptr = off)
  int dbg_step;
  // DDP across ranks (world > 1): per-step gradient exchange through the LL
  // slots of a dedicated p2p buffer set (csrc/p2p_allreduce.hip)
  int rank, world;
  unsigned long long* peer_ll[8];   // each rank's LL slot array [2][world][slot_elems]
  const unsigned long long* local_ll;
  long long slot_elems;
  int* xepoch;                      // exchange epoch counter (device, advanced by nsteps)
  int* xerr;                        // raised when a peer never delivered (bounded wait)
  int timeout_iters;
  int xmode;                        // 1: one-shot (every gradient to every rank), 2: reduce-scatter to the
                                    // owner rank (j % world) + all-gather of the summed gradient,
                                    // 3: helper workgroups run the one-shot exchange (grid 1 + nh)
  // xmode 3: gradients leave the loop's CU once (xg_out, fragment order), nh helper
  // workgroups push / reduce them across ranks on their own CUs, sums come back in xg_red
  float* xg_out;                    // [2][xe]
  float* xg_red;                    // [2][xe]
  int* xready;                      // [2][8 waves] epoch of each loop wave's gradients in xg_out[parity]
  int* xdone;                       // [nh] epoch each helper finished (helper h: elements [512 h, 512 h + 512))
  int nh, xe;
};

}  // namespace dta
