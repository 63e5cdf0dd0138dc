#!/bin/bash
# round 5, call J: in-step A/B of the GPT-2 GEMM picks the tracked table made from isolated timing
# (each variant forces one shape's implementation through a DTA_GEMM_CACHE override; two rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
run() {  # run <tag> <json overrides>
  echo "$2" > /tmp/ov_$1.json
  DTA_GEMM_CACHE=/tmp/ov_$1.json bash $S lm j_$1 --model gpt2 --strategy ddp --steps 30 --warmup 5 > /dev/null || return 1
  python3 -c "import json,sys; j=json.loads(open('gpurun_out/lm_j_$1.json').read().strip().splitlines()[-1]); print(json.dumps({'tag':'$1','ms':j['ms_per_step']}))" | tee -a gpurun_out/gemm_ab_r5j.jsonl
}
: > gpurun_out/gemm_ab_r5j.jsonl
for r in 1 2; do
  run base_$r '{}' &&
  run dgelu_t7_$r '{"dgelu 8192x3072x768": 17}' &&
  run dgelu_t6_$r '{"dgelu 8192x3072x768": 16}' &&
  run dgelu_lib_$r '{"dgelu 8192x3072x768": 0}' &&
  run dgrad_t3_$r '{"dgrad 8192x768x2304": 13, "dgrad 8192x768x3072": 13, "dgrad 8192x768x768": 13}' &&
  run dgrad_t6_$r '{"dgrad 8192x768x2304": 16, "dgrad 8192x768x3072": 16, "dgrad 8192x768x768": 16}' &&
  run fwdb_t7_$r '{"fwdb 8192x2304x768": 17, "fwdb 8192x768x3072": 17}' &&
  run fwdgelu_t3_$r '{"fwd_gelub 8192x3072x768": 13}' &&
  run fwdgelu_t7_$r '{"fwd_gelub 8192x3072x768": 17}' || exit 1
done
