#!/bin/bash
# round 5, call I: HEAD validation -- whole GPU suite, smoke, benches, config 5 through the entrypoint,
# step profiles, headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
: > gpurun_out/attn_diag_r5i.jsonl
for r in 1 2; do
  for b in u3 u4 hot; do
    timeout -k 10 120 ./scripts/attn_diag_$b "$b" >> gpurun_out/attn_diag_r5i.jsonl || exit $?
  done
done
cat gpurun_out/attn_diag_r5i.jsonl
bash $S tests && bash $S smoke &&
bash $S lm g2i --model gpt2 --strategy ddp --steps 30 --warmup 5 &&
bash $S lm g2i_fsdp --model gpt2 --strategy fsdp --steps 30 --warmup 5 &&
bash $S lm lli --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S prof lli bench_lm.py --model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2 &&
bash $S prof g2i bench_lm.py --model gpt2 --strategy ddp --steps 10 --warmup 3 &&
bash $S headline &&
timeout -k 10 600 torchrun --nproc_per_node=1 --master-addr 127.0.0.1 --master-port 29511 \
    src/multigpu_multi_node.py 2 0 model=llama3_8b train=llama3_8b_fsdp > gpurun_out/cfg5_r5i.log 2>&1 &&
grep -i "ms/step" gpurun_out/cfg5_r5i.log | tail -2
