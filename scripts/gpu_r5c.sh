#!/bin/bash
# round 5, call C: steps with the tracked GEMM table -- GPT-2 DDP (plain / optimizer in backward), Llama-3 8B
# FSDP, their rocprof kernel profiles, and one PMC pass over the Llama-shape attention kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S lm g2c --model gpt2 --strategy ddp --steps 20 --warmup 5 || exit $?
bash $S lm g2ovc --model gpt2 --strategy ddp --steps 20 --warmup 5 --overlap-opt || exit $?
bash $S lm llc --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 || exit $?
bash $S prof g2c python3 bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 || exit $?
bash $S prof llc python3 bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 || exit $?
bash $S pmc attn128 GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT \
    scripts/attn128_only.py 4 || exit $?
