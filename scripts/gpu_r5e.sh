#!/bin/bash
# round 5, call E: attention diagnostics (prefetch depth, backward ILV A/B, LDS-parity unrolled build u3),
# attention + LM-head GPU tests, GPT-2 head weight-gradient pick A/B in-step, row-blocked head + CE
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
: > gpurun_out/attn_diag_r5e.jsonl
for r in 1 2; do
  for b in pf3 u3; do
    for ilv in 0 1; do
      DTA_ATTN_BWD_ILV=$ilv timeout -k 10 120 ./scripts/attn_diag_$b "${b}_ilv${ilv}" >> gpurun_out/attn_diag_r5e.jsonl || exit $?
    done
  done
  DTA_ATTN_BWD_ILV=1 timeout -k 10 120 ./scripts/attn_diag_pf4 "pf4_ilv1" >> gpurun_out/attn_diag_r5e.jsonl || exit $?
  DTA_ATTN_BWD_ILV=0 timeout -k 10 120 ./scripts/attn_diag_nb3 "nb3_ilv0" >> gpurun_out/attn_diag_r5e.jsonl || exit $?
done
cat gpurun_out/attn_diag_r5e.jsonl
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_lm_ops_gpu.py -k "attention or cross_entropy or fused_model or chunked" > gpurun_out/pytest_r5e.log 2>&1 \
  || { tail -30 gpurun_out/pytest_r5e.log; exit 1; }
tail -1 gpurun_out/pytest_r5e.log
for r in 1 2; do
  bash $S lm g2e_w4_$r --model gpt2 --strategy ddp --steps 30 --warmup 5 || exit $?
  DTA_GEMM_CACHE=scripts/gemm_override_headwgrad_lib.json bash $S lm g2e_lib_$r --model gpt2 --strategy ddp --steps 30 --warmup 5 || exit $?
done
bash $S lm g2e_ch2048 --model gpt2 --strategy ddp --steps 30 --warmup 5 --head-ce-chunk 2048 || exit $?
bash $S lm lle_ch0 --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 || exit $?
bash $S lm lle_ch4096 --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 --head-ce-chunk 4096 || exit $?
