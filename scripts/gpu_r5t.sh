#!/bin/bash
# round 5, call T: the stream-K forms of the k64 tiles -- correctness (exact / epilogues / busy chip, counters
# left zero), the tracked-table timing of every GPT-2 / Llama GEMM key with the stream-K candidates in, then a
# same-box in-step A/B of each model with the keys whose new isolated pick is a stream-K form
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
T=distributed_training_amd/ops/gemm_table_mi355x.json
bash $S tests tests/test_gemm64_gpu.py tests/test_lm_ops_gpu.py -k "stream_k or 192 or no_grad" &&
cp gpurun_out/pytest_gpu.log gpurun_out/pytest_gpu_r5t.log &&
bash $S table --only fwd,fwdb,fwd_gelub,dgrad,dgelu,wgrad,head_dgrad --merge $T --out gpurun_out/table_r5t.json &&
cp gpurun_out/gemm_table.jsonl gpurun_out/table_r5t.jsonl || exit 1
python3 - <<'PY' || exit 1
import json
e = json.load(open("gpurun_out/table_r5t.json"))["entries"]
ov_g, ov_l = {}, {}
for k, v in e.items():
    if v["pick_name"].endswith("sk"):
        dims = k.rsplit(" ", 1)[1].split("x")
        llama = any(d in ("4096", "14336", "6144", "28672", "128256") for d in dims)
        (ov_l if llama else ov_g)[k] = v["pick"]
json.dump(ov_g, open("/tmp/ov_sk_g.json", "w"))
json.dump(ov_l, open("/tmp/ov_sk_l.json", "w"))
print(json.dumps({"gpt2": ov_g, "llama": ov_l}))
PY
: > gpurun_out/ab_sk_r5t.jsonl
run() {  # run <tag> <env> <model args...>
  local tag=$1 ev=$2; shift 2
  env $ev bash $S lm t_$tag "$@" > /dev/null || return 1
  python3 -c "import json; j=json.loads(open('gpurun_out/lm_t_$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag':'$tag','ms':j['ms_per_step']}))" | tee -a gpurun_out/ab_sk_r5t.jsonl
}
G="--model gpt2 --strategy ddp --steps 30 --warmup 5"
L="--model llama3_8b --strategy fsdp --batch 1 --seq 8192 --steps 6 --warmup 2"
for r in 1 2; do
  run g_base_$r "DTA_X=0" $G && run g_sk_$r "DTA_GEMM_CACHE=/tmp/ov_sk_g.json" $G || exit 1
done
for r in 1 2; do
  run l_base_$r "DTA_X=0" $L && run l_sk_$r "DTA_GEMM_CACHE=/tmp/ov_sk_l.json" $L || exit 1
done
