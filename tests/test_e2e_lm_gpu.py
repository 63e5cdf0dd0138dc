"""The transformer configs through the reference-compatible torchrun entrypoint
``src/multigpu_multi_node.py`` on ONE GPU (world size 1), shrunk by overrides: the Llama FSDP
config with the whole-step hipGraph (``train.step_graph``: at one rank every FSDP unit aliases its
shard, parallel/fsdp.py ``graph_capturable``) and the GPT-2 DDP config (step graph on in its yaml)
-- the step is captured (the trainer's log line), the loss is finite and falls, the snapshot is
written and a resumed run continues from it.  CPU counterparts with two gloo ranks:
tests/test_e2e_lm_cpu.py."""
import os
import re
import socket
import subprocess
import sys

import pytest
import torch

from tests.test_e2e_lm_cpu import ENTRY, ROOT, TINY_GPT2, TINY_LLAMA

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp_path, tag, args, epochs):
    snap = tmp_path / "snap.pt"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node=1", "--master-addr=127.0.0.1",
           f"--master-port={_port()}", ENTRY, str(epochs), "1", *args, "train.device=cuda", "train.save_every=1",
           f"hydra.run.dir={tmp_path}/{tag}", f"train.snapshot_path={snap}"]
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return snap, (tmp_path / tag / "train.log").read_text()


def _losses(log):
    vals = [float(x) for x in re.findall(r"samples/s \| loss ([0-9.naif]+)", log)]
    assert vals and all(v == v and v < 1e9 for v in vals), vals
    return vals


# the GPU attention kernels take head dims 64 / 128: the CPU tests' 64-wide models widened to 256 (4 heads)
GPU_WIDTH = ["model.n_embd=256"]


@pytest.mark.parametrize("name,args", [
    ("llama_fsdp", TINY_LLAMA + GPU_WIDTH + ["model.ffn_hidden=512", "train=llama3_8b_fsdp", "train.step_graph=true",
                                             "train.dataset_size=64"]),
    ("gpt2_ddp", TINY_GPT2 + GPU_WIDTH + ["train=gpt2_ddp", "train.dataset_size=128"]),
])
def test_lm_step_graph_through_entrypoint_gpu(tmp_path, name, args):
    snap, log = _run(tmp_path, "run", args, epochs=4)
    assert "0] Running with 1 processes total" in log, log[-2000:]
    assert "whole training step is replayed as one hipGraph" in log, log[-3000:]
    assert "step graph disabled" not in log
    losses = _losses(log)
    assert len(losses) == 4 and losses[-1] < losses[0], losses
    ck = torch.load(snap, weights_only=True)
    assert ck["EPOCHS_RUN"] == 3
    for v in ck["MODEL_STATE"].values():
        assert torch.isfinite(v.float()).all()
    _, log2 = _run(tmp_path, "run2", args, epochs=5)
    assert "Loading snapshot" in log2 and "0] Epoch 1 |" not in log2
    resumed = _losses(log2)
    assert resumed[0] < losses[0]


@pytest.mark.parametrize("name,args", [
    ("gpt2_fsdp", TINY_GPT2 + GPU_WIDTH + ["train=gpt2_fsdp", "train.dataset_size=128"]),
    ("llama_fsdp", TINY_LLAMA + GPU_WIDTH + ["model.ffn_hidden=512", "train=llama3_8b_fsdp", "train.dataset_size=64"]),
    ("gpt2_ddp", TINY_GPT2 + GPU_WIDTH + ["train=gpt2_ddp", "train.dataset_size=128"]),
])
def test_lm_step_graph_two_ranks_through_entrypoint(tmp_path, name, args):
    """Two ranks sharing the GPU (DTA_SHARED_GPU=1: the IPC data plane, gloo control plane) through the
    entrypoint: the Trainer's capture policy (engine/step_graph.py) sees every collective on the IPC plane and
    replays the whole step -- FSDP FULL_SHARD included, its units gathered into the fixed ring buffers
    (parallel/fsdp.py _GatherRing) -- on both ranks; the loss is finite and falls."""
    tag = "ws2"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           f"--master-port={_port()}", ENTRY, "3", "1000", *args, "train.device=cuda",
           f"hydra.run.dir={tmp_path}/{tag}", f"train.snapshot_path={tmp_path / 'snap.pt'}"]
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="4", DTA_SHARED_GPU="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    log = (tmp_path / tag / "train.log").read_text()
    assert "Running with 2 processes total" in log, log[-2000:]
    assert log.count("whole training step is replayed as one hipGraph") == 2, log[-3000:]
    assert "step graph disabled" not in log and "step graph not used" not in log
    losses = _losses(log)  # (both ranks log each epoch: first two lines epoch 0, last two the final epoch)
    assert len(losses) == 6 and sum(losses[-2:]) < sum(losses[:2]), losses
