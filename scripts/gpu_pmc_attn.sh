#!/bin/bash
# Effective clock / wave occupancy of the attention kernels in isolation vs inside
# the Llama-3 8B step (GRBM_GUI_ACTIVE / 8 / kernel time = clock, MI355X_MICROARCH.md).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/pmc_attn gpurun_out/pmc_llama
CTRS="GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"
timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc_attn -o run -- \
  python3 scripts/bench_attn.py llama8b > gpurun_out/pmc_attn/log 2>&1
timeout -s KILL 400 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc_llama -o run -- \
  python3 bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 1 --warmup 1 > gpurun_out/pmc_llama/log 2>&1
ls gpurun_out/pmc_attn gpurun_out/pmc_llama
