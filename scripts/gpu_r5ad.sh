#!/bin/bash
# round 5, call AD: last full GPU suite + smoke + headline at the final HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S tests && cp gpurun_out/pytest_gpu.log gpurun_out/pytest_gpu_r5ad.log && bash $S smoke && bash $S headline
