#!/bin/bash
# round 5, call G: benches + step profiles at HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S lm g2g --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
bash $S lm llg --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S prof g2g bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 &&
bash $S prof llg bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S headline
