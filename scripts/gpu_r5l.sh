#!/bin/bash
# round 5, call L: in-step A/B of the Llama-3 8B GEMM picks with small isolated-timing margins
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
run() {  # run <tag> <json overrides>
  echo "$2" > /tmp/ov_$1.json
  DTA_GEMM_CACHE=/tmp/ov_$1.json bash $S lm l_$1 --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 > /dev/null || return 1
  python3 -c "import json,sys; j=json.loads(open('gpurun_out/lm_l_$1.json').read().strip().splitlines()[-1]); print(json.dumps({'tag':'$1','ms':j['ms_per_step']}))" | tee -a gpurun_out/gemm_ab_r5l.jsonl
}
: > gpurun_out/gemm_ab_r5l.jsonl
for r in 1 2; do
  run base_$r '{}' &&
  run wg6144_t5_$r '{"wgrad 6144x4096x8192": 15}' &&
  run dg_lib_$r '{"dgrad 8192x4096x4096": 0, "dgrad 8192x4096x6144": 0}' &&
  run hd_t10_$r '{"head_dgrad 8192x4096x128256": 20, "head_wgrad 128256x4096x8192": 20}' || exit 1
done
