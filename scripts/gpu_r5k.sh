#!/bin/bash
# round 5, call K: caching-allocator A/B (expandable segments) on the LM steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
for r in 1 2; do
  bash $S lm k_g2_def_$r --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
  PYTORCH_HIP_ALLOC_CONF=expandable_segments:True bash $S lm k_g2_exp_$r --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
  bash $S lm k_ll_def_$r --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
  PYTORCH_HIP_ALLOC_CONF=expandable_segments:True bash $S lm k_ll_exp_$r --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 || exit 1
done
