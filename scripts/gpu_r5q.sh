#!/bin/bash
# round 5, call Q: deferred norm gamma / beta gradients (one batched column-sum launch per flush) -- the
# engine / model / norm GPU tests, then same-box A/B (DTA_NORM_DEFER=0 vs default) on GPT-2 DDP / FSDP and Llama
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S tests tests/test_lm_ops_gpu.py tests/test_engine_gpu.py tests/test_e2e_lm_gpu.py tests/test_ipc_gpu.py &&
for r in 1 2; do
  bash $S lm q_g2_on_$r --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
  DTA_NORM_DEFER=0 bash $S lm q_g2_off_$r --model gpt2 --strategy ddp --steps 30 --warmup 5 || exit 1
done &&
bash $S lm q_g2f_on --model gpt2 --strategy fsdp --steps 30 --warmup 5 &&
DTA_NORM_DEFER=0 bash $S lm q_g2f_off --model gpt2 --strategy fsdp --steps 30 --warmup 5 &&
bash $S lm q_ll_on --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
DTA_NORM_DEFER=0 bash $S lm q_ll_off --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S prof g2q bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3
