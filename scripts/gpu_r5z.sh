#!/bin/bash
# round 5, call Z: final-HEAD validation (after TunableOp, the stream-K / 192 tiles and the k64 TU split) -- full GPU suite, smoke, headline bench, GPT-2 DDP / FSDP and Llama-3 8B
# benches, both step profiles, config 5 through the reference entrypoint
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S tests && cp gpurun_out/pytest_gpu.log gpurun_out/pytest_gpu_r5z.log &&
bash $S smoke &&
bash $S headline &&
bash $S lm g2z --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
bash $S lm g2z_fsdp --model gpt2 --strategy fsdp --steps 30 --warmup 5 &&
bash $S lm llz --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S prof llz bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S prof g2z bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 &&
timeout -k 10 600 torchrun --nproc_per_node=1 --master-addr 127.0.0.1 --master-port 29511 \
    src/multigpu_multi_node.py 2 0 model=llama3_8b train=llama3_8b_fsdp > gpurun_out/cfg5_r5z.log 2>&1 &&
grep -i "ms/step" gpurun_out/cfg5_r5z.log | tail -2
