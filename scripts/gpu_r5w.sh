#!/bin/bash
# round 5, call W: the tracked TunableOp results loaded by the framework itself (ops/lm.py _library_tuning) --
# GPT-2 DDP with them (default) vs DTA_TUNABLEOP=0, same box; the LM GPU tests with them in; no results file
# may be written by a run (tuning off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
bash $S tests tests/test_lm_ops_gpu.py tests/test_e2e_lm_gpu.py tests/test_engine_gpu.py || exit 1
G="--model gpt2 --strategy ddp --steps 30 --warmup 5"
: > gpurun_out/ab_tunableop_r5w.jsonl
run() {  # run <tag> <env> <model args...>
  local tag=$1 ev=$2; shift 2
  env $ev bash $S lm w_$tag "$@" > /dev/null || return 1
  python3 -c "import json; j=json.loads(open('gpurun_out/lm_w_$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag':'$tag','ms':j['ms_per_step']}))" | tee -a gpurun_out/ab_tunableop_r5w.jsonl
}
for r in 1 2 3; do
  run g_off_$r "DTA_TUNABLEOP=0" $G && run g_on_$r "DTA_X=0" $G || exit 1
done
run g_fsdp_on "DTA_X=0" --model gpt2 --strategy fsdp --steps 30 --warmup 5 &&
find . -name "tunableop_results*" | tee gpurun_out/tunableop_stray_files.txt
