# bench.py's driver-style 1-GPU run in fresh processes, with the timed call's host time traced
export PYTHONPATH=$PWD DTA_BENCH_TRACE=1
for i in 1 2 3; do timeout -k 10 100 python bench.py --steps 20 --warmup 5 2>&1 | grep -o '\[bench\].*\|\[fused_mlp\].*\|"value": [0-9.]*' | tr '\n' ' '; echo; done
for i in 1 2; do DTA_SYNC_SPIN=0 timeout -k 10 100 python bench.py --steps 20 --warmup 5 2>&1 | grep -o '\[bench\].*\|"value": [0-9.]*' | tr '\n' ' '; echo; done
