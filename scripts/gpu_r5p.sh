#!/bin/bash
# round 5, call P: final-HEAD step profiles (in-step table overrides: Llama head forward on k64, GPT-2 dGELU
# t7 and N = 768 input gradients t6) + benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S lm g2p --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
bash $S lm g2p_fsdp --model gpt2 --strategy fsdp --steps 30 --warmup 5 &&
bash $S lm llp --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S prof llp bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S prof g2p bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 &&
timeout -k 10 600 torchrun --nproc_per_node=1 --master-addr 127.0.0.1 --master-port 29511 \
    src/multigpu_multi_node.py 2 0 model=llama3_8b train=llama3_8b_fsdp > gpurun_out/cfg5_r5p.log 2>&1 &&
grep -i "ms/step" gpurun_out/cfg5_r5p.log | tail -2
