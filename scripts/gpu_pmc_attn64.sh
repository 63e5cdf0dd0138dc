#!/bin/bash
# PMC passes over the GPT-2-shape (D = 64) attention kernels: where the cycles go
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1)); mkdir -p gpurun_out/pmc64_$i
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc64_$i -o run -- python3 scripts/attn64_only.py > gpurun_out/pmc64_$i/log 2>&1
done
find gpurun_out/pmc64_1 gpurun_out/pmc64_2 -name "*counter_collection.csv" | head
