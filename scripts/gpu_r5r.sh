#!/bin/bash
# round 5, call R: the 192-wide k64 tiles (11 = 256 x 192, 12 = 128 x 192; K-major operands) -- correctness,
# isolated timing of every forward GEMM key against hipBLASLt and the other tiles, then a same-box in-step A/B
# of GPT-2 DDP with each GPT-2 forward key forced to its fastest 192-wide tile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=scripts/gpu.sh
T=distributed_training_amd/ops/gemm_table_mi355x.json
bash $S tests tests/test_gemm64_gpu.py &&
bash $S table --only fwd,fwdb,fwd_gelub,head_fwd --merge $T --out gpurun_out/table_r5r.json &&
cp gpurun_out/gemm_table.jsonl gpurun_out/table_r5r.jsonl || exit 1
python3 - <<'PY' || exit 1
import json
e = json.load(open("gpurun_out/table_r5r.json"))["entries"]
ov = {}
for k, v in e.items():
    M = k.rsplit(" ", 1)[1].split("x")
    if M[2] not in ("768", "3072") or not k.startswith(("fwd", "head_fwd")):
        continue  # the GPT-2 forward keys
    c = {t: v["us"][t] for t in ("k64/t11", "k64/t12") if t in v["us"]}
    if c:
        best = min(c, key=c.get)
        ov[k] = 10 + int(best.split("t")[-1])
json.dump(ov, open("/tmp/ov192.json", "w"))
print(json.dumps(ov))
PY
: > gpurun_out/ab192_r5r.jsonl
run() {  # run <tag> [env]: GPT-2 DDP, one bench
  env $2 bash $S lm r_$1 --model gpt2 --strategy ddp --steps 30 --warmup 5 > /dev/null || return 1
  python3 -c "import json; j=json.loads(open('gpurun_out/lm_r_$1.json').read().strip().splitlines()[-1]); print(json.dumps({'tag':'$1','ms':j['ms_per_step']}))" | tee -a gpurun_out/ab192_r5r.jsonl
}
for r in 1 2; do
  run base_$r "DTA_X=0" && run t192_$r "DTA_GEMM_CACHE=/tmp/ov192.json" || exit 1
done
