#!/bin/bash
# attention kernels: numerics tests, GPT-2 / Llama shape timings, one PMC pass over D = 64
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_lm_ops_gpu.py tests/test_fuzz_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" 2>&1 | tail -2
timeout -k 10 200 python scripts/bench_attn.py gpt2 llama8b | cut -c1-200
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
mkdir -p gpurun_out/pmc64_3
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc64_3 -o run -- python3 scripts/attn64_only.py > gpurun_out/pmc64_3/log 2>&1
