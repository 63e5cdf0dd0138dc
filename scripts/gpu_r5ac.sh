#!/bin/bash
# round 5, call AC: the tracked GEMM table extended to GPT-2 at B = 16 and 32 (the keys missing from it, every
# candidate timed as for the B = 8 keys), then both batch sizes benched with the extended table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
T=distributed_training_amd/ops/gemm_table_mi355x.json
bash $S table --gpt2-batches 8,16,32 --new-only --merge $T --out gpurun_out/table_r5ac.json &&
cp gpurun_out/gemm_table.jsonl gpurun_out/table_r5ac.jsonl &&
cp gpurun_out/table_r5ac.json $T &&
bash $S lm ac_g16 --model gpt2 --strategy ddp --batch 16 --steps 20 --warmup 5 &&
bash $S lm ac_g32 --model gpt2 --strategy ddp --batch 32 --steps 20 --warmup 5 &&
python3 -c "
import json
for f in ('lm_ac_g16', 'lm_ac_g32'):
    j = json.loads(open('gpurun_out/%s.json' % f).read().strip().splitlines()[-1])
    print(f, j['ms_per_step'], sorted(set(j.get('gemm_pick_source', {}).values())))
"
