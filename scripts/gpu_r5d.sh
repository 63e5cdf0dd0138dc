#!/bin/bash
# round 5, call D: attention numerics (interleaved dK/dV softmax), attention A/B, GPT-2 GEMM table A/B,
# step profiles, one attention PMC pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_lm_ops_gpu.py -k "attention" > gpurun_out/pytest_r5d.log 2>&1 || { tail -30 gpurun_out/pytest_r5d.log; exit 1; }
tail -2 gpurun_out/pytest_r5d.log
: > gpurun_out/attn_ab_r5d.jsonl
for r in 1 2; do
  for ilv in 0 1; do
    DTA_ATTN_DKDV_ILV=$ilv timeout -k 10 300 python scripts/bench_attn.py llama8b gpt2 | sed "s/^{/{\"dkdv_ilv\": $ilv, /" >> gpurun_out/attn_ab_r5d.jsonl || exit $?
  done
done
cut -c1-200 gpurun_out/attn_ab_r5d.jsonl
for r in 1 2; do
  DTA_GEMM_TABLE=0 bash $S lm g2_notable_$r --model gpt2 --strategy ddp --steps 20 --warmup 5 || exit $?
  bash $S lm g2_table_$r --model gpt2 --strategy ddp --steps 20 --warmup 5 || exit $?
done
bash $S prof g2d bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 || exit $?
DTA_GEMM_TABLE=0 bash $S prof g2d_notable bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 || exit $?
bash $S prof lld bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 || exit $?
bash $S pmc attn128 GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT \
    scripts/attn128_only.py 4 || exit $?
