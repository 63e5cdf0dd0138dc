#!/bin/bash
# round 5, call A: GEMM epilogue diagnostics, GPU test suite, BASELINE config 5 through the reference entrypoint
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for d in 0 1 2; do
  timeout -k 10 120 ./scripts/k64_epi_$d >> gpurun_out/k64_epi_diag.jsonl 2>&1 || exit $?
done
timeout -k 10 120 python scripts/torch_mm_times.py >> gpurun_out/k64_epi_diag.jsonl 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_r5a.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_r5a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 torchrun --nproc_per_node=1 --master-addr 127.0.0.1 --master-port 29511 \
    src/multigpu_multi_node.py 2 0 model=llama3_8b train=llama3_8b_fsdp > gpurun_out/cfg5_r5a.log 2>&1
echo "cfg5 rc=$?" >> gpurun_out/cfg5_r5a.log
