"""The bench.py / bench_lm.py JSON-line contract the round driver parses (one
line on rank 0; metric / config of BASELINE.json; timing fields consistent)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _run(args, timeout=240):
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    p = subprocess.run([sys.executable, *args], cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_headline_json_line():
    base = json.loads((ROOT / "BASELINE.json").read_text())
    out = _run(["bench.py", "--steps", "128", "--warmup", "16"])
    assert out["metric"] == base["metric"]
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == 1 and out["steps"] == 128 and out["warmup"] == 16
    assert out["higher_is_better"] is True and out["scaling"] == "weak" and out["dtype"] == "bf16"
    # value = whole-job samples/s = global batch / step time
    gb = out["config"]["global_batch"]
    assert abs(out["value"] - gb / (out["ms_per_step"] * 1e-3)) / out["value"] < 0.02
    assert out["config"]["parallelism"] == "dp1"


def test_bench_lm_json_line():
    out = _run(["bench_lm.py", "--model", "gpt2", "--strategy", "ddp", "--steps", "3", "--warmup", "1"])
    assert out["metric"].startswith("tokens/s") and out["value"] > 0 and out["n_gpus"] == 1
    assert out["config"]["model"] == "gpt2" and out["config"]["seq_len"] == 1024


def _torchrun(n, args, timeout=420):
    from dist_utils import free_port

    env = dict(os.environ, PYTHONPATH=str(ROOT), DTA_SHARED_GPU="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), *args]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_multi_rank_shared_gpu():
    """The driver's N-GPU command (torchrun, one JSON line from rank 0), rehearsed with
    4 ranks on this box's one GPU: calibration of the DDP step forms, in-kernel
    exchange, MAX-over-ranks timing."""
    out = _torchrun(4, ["bench.py", "--gpus", "4", "--steps", "20", "--warmup", "5"])
    assert out["n_gpus"] == 4 and out["steps"] == 20 and out["warmup"] == 5
    assert out["config"]["parallelism"] == "dp4" and out["config"]["global_batch"] == 128
    assert out["value"] > 0 and "shared_gpu" in out
    assert out["calibration_ms"], out  # every step form was timed on the node


@pytest.mark.parametrize("strategy", ["ddp", "fsdp"])
def test_bench_lm_two_ranks_shared_gpu(strategy):
    out = _torchrun(2, ["bench_lm.py", "--gpus", "2", "--model", "llama_tiny", "--strategy", strategy,
                        "--batch", "2", "--seq", "256", "--steps", "3", "--warmup", "1"])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["comm"] == "IpcComm"
    assert out["final_loss"] == out["final_loss"]  # finite
