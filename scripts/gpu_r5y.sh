#!/bin/bash
# round 5, call Y: attention at HEAD -- standalone timing of both shapes (bench_attn.py, vs torch SDPA) and one PMC
# pass per shape (MFMA busy, wait / wait-inst / active shares, LDS bank conflicts)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
timeout -k 10 300 python scripts/bench_attn.py gpt2 llama8b > gpurun_out/attn_bench_r5y.jsonl 2> gpurun_out/attn_bench_r5y.err &&
cut -c1-300 gpurun_out/attn_bench_r5y.jsonl &&
bash $S pmc attn64 GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT \
    scripts/attn64_only.py &&
bash $S pmc attn128 GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT \
    scripts/attn128_only.py 4
