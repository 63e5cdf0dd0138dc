#!/bin/bash
# round 5, call B: measure the tracked GEMM table; re-run the two tests fixed after call A
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu.sh table --out gpurun_out/gemm_table_mi355x.json || exit $?
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_e2e_lm_gpu.py::test_lm_step_graph_through_entrypoint_gpu" \
  "tests/test_lm_ops_gpu.py::test_ddp_linear_gradients_written_into_flat_buffer" \
  "tests/test_lm_ops_gpu.py::test_ddp_deferred_grouped_weight_gradients" > gpurun_out/pytest_r5b.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_r5b.log
