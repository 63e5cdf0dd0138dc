#!/bin/bash
# Same-box A/B of the GPT-2 DDP step: head weight-gradient scale on the [V, C] product (B, current) vs on the [N, C] operand (A).
set -uo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
cp distributed_training_amd/ops/lm.py /tmp/lm_B.py
sed "s/dw = gemm(dlogits, x2, True, True, kind=\"head_wgrad\", out=_grad_dest(ctx.wparam)).mul_(s)/dw = gemm(dlogits, x2 * s, True, True, kind=\"head_wgrad\", out=_grad_dest(ctx.wparam))/" /tmp/lm_B.py > /tmp/lm_A.py
grep -c "x2 \* s, True" /tmp/lm_A.py
: > gpurun_out/ab_heads.txt
for i in 1 2 3; do for v in A B; do
  cp /tmp/lm_$v.py distributed_training_amd/ops/lm.py
  timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --json-out /tmp/r.json > /dev/null 2>&1 || exit 1
  python -c "import json; d=json.load(open('/tmp/r.json')); print('$v', d['ms_per_step'], d['final_loss'])" >> gpurun_out/ab_heads.txt
done; done
cp /tmp/lm_B.py distributed_training_amd/ops/lm.py
cat gpurun_out/ab_heads.txt
