#!/bin/bash
# round 5, call M: final-HEAD validation (GPU suite, smoke, benches, headline) and a cross-box check of the
# tracked GEMM table (re-measured here, picks compared)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S tests && bash $S smoke &&
bash $S lm g2m --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
bash $S lm llm --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S headline &&
bash $S table --check distributed_training_amd/ops/gemm_table_mi355x.json
