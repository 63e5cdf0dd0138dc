#!/bin/bash
# round 5, call S: full GPU suite + smoke at HEAD (192-wide tiles in), shared-GPU rehearsal of bench.py at
# 2 / 4 ranks, and a same-box in-step A/B of the GPT-2 forward keys whose isolated best is a 192-wide tile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S tests && bash $S smoke &&
bash $S shared 2 b2 bench.py --gpus 2 --steps 200 --warmup 20 &&
bash $S shared 4 b4 bench.py --gpus 4 --steps 200 --warmup 20 || exit 1
echo '{"fwd_gelub 8192x3072x768": 22}' > /tmp/ovA.json
echo '{"fwd_gelub 8192x3072x768": 22, "fwdb 8192x2304x768": 22}' > /tmp/ovB.json
: > gpurun_out/ab192_r5s.jsonl
run() {  # run <tag> [env]: GPT-2 DDP, one bench
  env $2 bash $S lm s_$1 --model gpt2 --strategy ddp --steps 30 --warmup 5 > /dev/null || return 1
  python3 -c "import json; j=json.loads(open('gpurun_out/lm_s_$1.json').read().strip().splitlines()[-1]); print(json.dumps({'tag':'$1','ms':j['ms_per_step']}))" | tee -a gpurun_out/ab192_r5s.jsonl
}
for r in 1 2; do
  run base_$r "DTA_X=0" && run gelu192_$r "DTA_GEMM_CACHE=/tmp/ovA.json" && run gelu_qkv192_$r "DTA_GEMM_CACHE=/tmp/ovB.json" || exit 1
done
