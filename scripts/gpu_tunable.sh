set -euo pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/tunable
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunable/gpt2_%d.csv
timeout -k 10 600 python bench_lm.py --model gpt2 --strategy ddp --steps 20 --warmup 5 > gpurun_out/tunable/tune.json 2> gpurun_out/tunable/tune.err
cat gpurun_out/tunable/tune.json
export PYTORCH_TUNABLEOP_TUNING=0
timeout -k 10 300 python bench_lm.py --model gpt2 --strategy ddp --steps 20 --warmup 5 > gpurun_out/tunable/use.json 2> gpurun_out/tunable/use.err
cat gpurun_out/tunable/use.json
