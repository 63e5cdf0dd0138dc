#!/bin/bash
# round 5, call AA: GPT-2 small at B = 32 x 1024 (DDP and FSDP) at the final HEAD -- the larger-batch row of the
# README table (round 4's 969 K tokens/s)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S lm aa_g32 --model gpt2 --strategy ddp --batch 32 --steps 20 --warmup 5 &&
bash $S lm aa_g32_fsdp --model gpt2 --strategy fsdp --batch 32 --steps 20 --warmup 5
