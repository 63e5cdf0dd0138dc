#!/bin/bash
# round 5, call F: whole GPU test suite + smoke on the HEAD extension (LDS-parity unrolled attention,
# per-D backward ILV default, CE row kernel with 4 loads in flight, row-blocked head + CE)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu.sh tests && bash scripts/gpu.sh smoke
