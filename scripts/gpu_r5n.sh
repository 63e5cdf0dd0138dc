#!/bin/bash
# round 5, call N: the row-blocked LM head + CE with its weight gradient written into the final slice in the
# forward -- peak memory and step time against the one-block head, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S lm n_g2_ch0 --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
bash $S lm n_g2_ch2048 --model gpt2 --strategy ddp --steps 30 --warmup 5 --head-ce-chunk 2048 &&
bash $S lm n_g2_ch4096 --model gpt2 --strategy ddp --steps 30 --warmup 5 --head-ce-chunk 4096 &&
bash $S lm n_ll_ch0 --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S lm n_ll_ch2048 --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 --head-ce-chunk 2048 &&
bash $S lm n_ll_ch4096 --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 --head-ce-chunk 4096 || exit 1
run() {  # run <tag> <json overrides>: Llama forwards on the hand-written tile instead of hipBLASLt, in the step
  echo "$2" > /tmp/ov_$1.json
  DTA_GEMM_CACHE=/tmp/ov_$1.json bash $S lm n_$1 --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 > /dev/null || return 1
  python3 -c "import json,sys; j=json.loads(open('gpurun_out/lm_n_$1.json').read().strip().splitlines()[-1]); print(json.dumps({'tag':'$1','ms':j['ms_per_step']}))" | tee -a gpurun_out/gemm_ab_r5n.jsonl
}
: > gpurun_out/gemm_ab_r5n.jsonl
for r in 1 2; do
  run base_$r '{}' &&
  run fwd_t5_$r '{"fwd 8192x4096x4096": 15, "fwd 8192x6144x4096": 15, "fwd 8192x28672x4096": 15, "fwd 8192x4096x14336": 15}' &&
  run headfwd_t5_$r '{"head_fwd 8192x128256x4096": 15}' || exit 1
done
