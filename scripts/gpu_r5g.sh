#!/bin/bash
# round 5, call G: benches + step profiles at HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S tests tests/test_lm_ops_gpu.py -k "norm or cross_entropy or fused_model" &&
bash $S lm g2g --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
bash $S lm llg --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S prof g2g bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 &&
bash $S prof llg bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S headline &&
timeout -k 10 600 torchrun --nproc_per_node=1 --master-addr 127.0.0.1 --master-port 29511 \
    src/multigpu_multi_node.py 2 0 model=llama3_8b train=llama3_8b_fsdp > gpurun_out/cfg5_r5g.log 2>&1 &&
grep -i "epoch\|ms/step\|checkpoint" gpurun_out/cfg5_r5g.log | tail -5
