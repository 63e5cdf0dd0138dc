#!/bin/bash
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/pmc_gemm1 gpurun_out/pmc_gemm2
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_gemm1 -o run -- python3 scripts/gemm_one.py 8192 4096 4096 1 > gpurun_out/pmc_gemm1/log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TA_TA_BUSY_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_gemm2 -o run -- python3 scripts/gemm_one.py 8192 4096 4096 1 > gpurun_out/pmc_gemm2/log 2>&1 || true
ls gpurun_out/pmc_gemm1 gpurun_out/pmc_gemm2
