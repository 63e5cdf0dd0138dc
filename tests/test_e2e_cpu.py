"""End-to-end runs of the reference-compatible entrypoints under torchrun (gloo, CPU)."""
import os
import re
import subprocess
import sys
from pathlib import Path

import pytest
import torch

from tests.dist_utils import free_port, run_gloo

ROOT = Path(__file__).resolve().parent.parent


def torchrun(args, nproc=2, extra=(), timeout=300, cwd=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", *extra, *args]
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=cwd or ROOT, env=env)


def test_legacy_entrypoint_ddp_mlp(tmp_path):
    snap = tmp_path / "snap.pt"
    r = torchrun([str(ROOT / "src" / "multigpu_multi_node.py"), "3", "1", "--batch_size", "16", "model=mlp2",
                  "train.loss=mse", "train.device=cpu", f"hydra.run.dir={tmp_path}/run", f"train.snapshot_path={snap}"])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    log = (tmp_path / "run" / "train.log").read_text()
    assert "[CPU0] Running with 2 processes total" in log and "[CPU1] Running with 2 processes total" in log
    assert "[CPU0] Epoch 2 | Batchsize: 16 | Steps: 64" in log
    assert "Epoch 2 | Training snapshot saved at" in log
    ck = torch.load(snap, weights_only=True)
    assert ck["EPOCHS_RUN"] == 2
    assert sorted(ck["MODEL_STATE"]) == ["module.fc1.bias", "module.fc1.weight", "module.fc2.bias",
                                         "module.fc2.weight"]
    # resume: the snapshot exists -> "Loading snapshot", training continues at EPOCHS_RUN
    r2 = torchrun([str(ROOT / "src" / "multigpu_multi_node.py"), "4", "1", "--batch_size", "16", "model=mlp2",
                   "train.loss=mse", "train.device=cpu", f"hydra.run.dir={tmp_path}/run2",
                   f"train.snapshot_path={snap}"])
    assert r2.returncode == 0, r2.stderr[-3000:]
    log2 = (tmp_path / "run2" / "train.log").read_text()
    assert "Loading snapshot" in log2
    assert "Epoch 1 |" not in log2 and "[CPU0] Epoch 2 | Batchsize" in log2 and "[CPU0] Epoch 3 | Batchsize" in log2
    assert torch.load(snap, weights_only=True)["EPOCHS_RUN"] == 3


def test_hydra_entrypoint_reference_default(tmp_path):
    """Reference default: Linear(20,1) + cross-entropy -> loss 0, weights unchanged."""
    snap = tmp_path / "s.pt"
    r = torchrun([str(ROOT / "src" / "distributed_trainer.py"), "train.total_epochs=1", "train.device=cpu",
                  f"hydra.run.dir={tmp_path}/run", f"train.snapshot_path={snap}", "train.seed=0"])
    assert r.returncode == 0, r.stderr[-3000:]
    ck = torch.load(snap, weights_only=True)
    assert sorted(ck["MODEL_STATE"]) == ["module.bias", "module.weight"]
    assert ck["EPOCHS_RUN"] == 0
    torch.manual_seed(0)
    lin = torch.nn.Linear(20, 1)
    torch.testing.assert_close(ck["MODEL_STATE"]["module.weight"], lin.weight.detach())


def test_fsdp_on_cpu_checkpoint(tmp_path):
    snap = tmp_path / "f.pt"
    r = torchrun([str(ROOT / "src" / "multigpu_multi_node.py"), "2", "1", "model=mlp2", "train.loss=mse",
                  "train.device=cpu", "train.parallel_strategy=fsdp", f"hydra.run.dir={tmp_path}/run",
                  f"train.snapshot_path={snap}"])
    assert r.returncode == 0, r.stderr[-3000:]
    ck = torch.load(snap, weights_only=True)
    assert sorted(ck["MODEL_STATE"]) == ["fc1.bias", "fc1.weight", "fc2.bias", "fc2.weight"]  # unprefixed
    assert ck["MODEL_STATE"]["fc1.weight"].shape == (512, 20)


def test_restart_after_injected_fault_resumes_from_snapshot(tmp_path):
    """Rank 1 dies mid-epoch (fault injection); the relaunched job (what
    ``torchrun --max-restarts`` or a cluster scheduler does) resumes from the
    last snapshot and finishes."""
    snap = tmp_path / "e.pt"
    args = [str(ROOT / "src" / "multigpu_multi_node.py"), "4", "1", "--batch_size", "64", "model=mlp2",
            "train.loss=mse", "train.device=cpu", f"hydra.run.dir={tmp_path}/run", f"train.snapshot_path={snap}"]
    r = torchrun(args + ["+train.fault_injection={rank: 1, epoch: 2, step: 3, kind: exit, code: 17}"])
    assert r.returncode != 0
    assert "fault injection" in r.stdout + r.stderr
    assert torch.load(snap, weights_only=True)["EPOCHS_RUN"] == 1
    r2 = torchrun(args)
    assert r2.returncode == 0, r2.stderr[-3000:]
    log = (tmp_path / "run" / "train.log").read_text()
    assert "Loading snapshot" in log
    assert torch.load(snap, weights_only=True)["EPOCHS_RUN"] == 3


def test_playground_manual_ddp(tmp_path):
    logdir = tmp_path / "logs"
    r = subprocess.run([sys.executable, str(ROOT / "src" / "playground" / "ddp_script.py"), "--world-size", "2",
                        "--epochs", "2", "--num-workers", "0", "--backend", "gloo", "--log-dir", str(logdir),
                        "--port", str(free_port())], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, PYTHONPATH=str(ROOT), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert r.returncode == 0, r.stderr[-3000:]
    logs = [(logdir / f"ddp_rank_{i}.log").read_text() for i in range(2)]

    def norms(text):
        return re.findall(r"Parameter: (\S+), (Gradient|Weight): (\S+)", text)

    n0, n1 = norms(logs[0]), norms(logs[1])
    assert len(n0) == len(n1) == 128  # 1000/2/32 -> 16 steps x 2 params x 2 lines x 2 epochs
    assert n0 == n1  # replicas stay identical
    assert "Average Loss" in logs[0]


def _desync(rank, ws):
    from distributed_training_amd.utils.desync import DesyncError, check_replicas_in_sync

    class Env:
        is_gpu = False
        local_rank = 0

    m = torch.nn.Linear(3, 2)
    with torch.no_grad():
        for p in m.parameters():
            p.fill_(1.0)
    check_replicas_in_sync(m, Env())
    if rank == 1:
        with torch.no_grad():
            m.bias.add_(1e-3)
    try:
        check_replicas_in_sync(m, Env())
    except DesyncError:
        return
    raise AssertionError("desync not detected")


def test_desync_detector():
    run_gloo(_desync, 2)
