#!/bin/bash
# round 5, call O: more GPT-2 in-step A/B (GEMM picks through DTA_GEMM_CACHE overrides, attention wave counts)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
run() {  # run <tag> <json overrides> [env assignments...]
  local tag=$1 ov=$2; shift 2
  echo "$ov" > /tmp/ov_$tag.json
  env "$@" DTA_GEMM_CACHE=/tmp/ov_$tag.json bash $S lm o_$tag --model gpt2 --strategy ddp --steps 30 --warmup 5 > /dev/null || return 1
  python3 -c "import json,sys; j=json.loads(open('gpurun_out/lm_o_$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag':'$tag','ms':j['ms_per_step']}))" | tee -a gpurun_out/gemm_ab_r5o.jsonl
}
: > gpurun_out/gemm_ab_r5o.jsonl
for r in 1 2; do
  run base_$r '{}' X=1 &&
  run proj_t6_$r '{"fwdb 8192x768x768": 16}' X=1 &&
  run proj_lib_$r '{"fwdb 8192x768x768": 0}' X=1 &&
  run hw_t8_$r '{"head_wgrad 50304x768x8192": 18}' X=1 &&
  run dgelu_t8_$r '{"dgelu 8192x3072x768": 18}' X=1 &&
  run dq8_$r '{}' DTA_ATTN_DQ_WAVES=8 &&
  run fwd4_$r '{}' DTA_ATTN_FWD_WAVES=4 || exit 1
done
