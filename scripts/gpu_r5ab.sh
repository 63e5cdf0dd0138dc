#!/bin/bash
# round 5, call AB: configurations off the tracked table (in-run candidate timing, stream-K among the
# candidates): GPT-2 at B = 16, Llama-3 8B at B = 2 x 4096
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S lm ab_g16 --model gpt2 --strategy ddp --batch 16 --steps 20 --warmup 5 &&
bash $S lm ab_ll2x4k --model llama3_8b --strategy fsdp --batch 2 --seq 4096 --steps 4 --warmup 2 &&
python3 -c "
import json
for f in ('lm_ab_g16', 'lm_ab_ll2x4k'):
    j = json.loads(open('gpurun_out/%s.json' % f).read().strip().splitlines()[-1])
    print(f, j['ms_per_step'], {k: v for k, v in j.get('gemm_impl', {}).items() if 'sk' in str(v) or 't11' in str(v) or 't12' in str(v)})
"
