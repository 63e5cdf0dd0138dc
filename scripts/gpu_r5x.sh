#!/bin/bash
# round 5, call X: the k64 GEMM split into csrc/gemm_k64_kernels.h + gemm_k64.hip + gemm_k64_sk.hip (parallel
# compile): the whole GEMM test file, smoke, and one GPT-2 / Llama bench each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S tests tests/test_gemm64_gpu.py tests/test_fused_linear_gpu.py && cp gpurun_out/pytest_gpu.log gpurun_out/pytest_gpu_r5x.log &&
bash $S smoke &&
bash $S lm x_g2 --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
bash $S lm x_ll --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2
