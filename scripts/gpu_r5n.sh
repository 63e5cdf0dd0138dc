#!/bin/bash
# round 5, call N: the row-blocked LM head + CE with its weight gradient written into the final slice in the
# forward -- peak memory and step time against the one-block head, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S lm n_g2_ch0 --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
bash $S lm n_g2_ch2048 --model gpt2 --strategy ddp --steps 30 --warmup 5 --head-ce-chunk 2048 &&
bash $S lm n_g2_ch4096 --model gpt2 --strategy ddp --steps 30 --warmup 5 --head-ce-chunk 4096 &&
bash $S lm n_ll_ch0 --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S lm n_ll_ch2048 --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 --head-ce-chunk 2048 &&
bash $S lm n_ll_ch4096 --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 --head-ce-chunk 4096
