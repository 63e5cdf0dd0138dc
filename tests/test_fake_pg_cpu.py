"""T3: the 8-rank node's sharding / bucketing arithmetic in ONE
process over torch's ``fake`` process group (collectives are no-ops, so only
shapes, padding, unit layout and the control flow of a step are checked; the
numerics at ws = 4 / 8 are covered over gloo in test_parallel_cpu.py)."""
import pytest
import torch
import torch.distributed as dist
import torch.nn.functional as F


@pytest.fixture
def fake_pg():
    from torch.testing._internal.distributed.fake_pg import FakeStore

    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    dist.init_process_group("fake", store=FakeStore(), rank=3, world_size=8)
    try:
        yield
    finally:
        dist.destroy_process_group()


def test_fsdp_units_at_world_8(fake_pg):
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.ops.optim import FusedAdamW
    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.fsdp import FullyShardedDataParallel

    torch.manual_seed(0)
    cfg = GPT2Config(n_layer=3, n_head=2, n_embd=40, vocab_size=101, block_size=16)
    m = GPT2(cfg)
    n_params = sum(p.numel() for p in m.parameters())
    fs = FullyShardedDataParallel(m, TorchComm(), torch.device("cpu"), wrap_policy={GPT2.block_class})
    assert fs.world_size == 8 and len(fs.units) == cfg.n_layer + 1  # blocks + root
    covered = 0
    for u in fs.units:
        assert u.total % (8 * 64) == 0 and u.shard_size * 8 == u.total  # 64-element (128-B bf16) aligned shards
        assert sum(u._split_sizes) == u.total
        assert all(o % 16 == 0 for o in u.offsets)  # every parameter 16-element aligned in the flat unit
        covered += sum(u.numels)
        assert not u.alias
    assert covered == n_params  # tied wte / lm_head counted once
    # this rank's shards: one flat master buffer of the summed shard sizes
    assert fs.shards.total >= sum(u.shard_size for u in fs.units)
    # a whole step runs through the unit hooks (no-op collectives: values are not checked)
    opt = FusedAdamW(fs.parameters(), lr=1e-3)
    x = torch.randint(0, 101, (2, 17))
    lo = fs(x[:, :-1])
    V = lo.shape[-1]  # vocabulary padded for the LM head
    assert lo.shape[:2] == (2, 16) and V >= 101
    F.cross_entropy(lo.reshape(-1, V), x[:, 1:].reshape(-1)).backward()
    opt.step()
    assert all(not u.gathered for u in fs.units if not u.is_root)  # resharded after backward


def test_ddp_buckets_at_world_8(fake_pg):
    from distributed_training_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_training_amd.parallel.comm import TorchComm
    from distributed_training_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    m = GPT2(GPT2Config(n_layer=4, n_head=2, n_embd=64, vocab_size=128, block_size=16))
    ddp = DistributedDataParallel(m, comm=TorchComm(), device=torch.device("cpu"), bucket_cap_mb=0.05,
                                  first_bucket_mb=0.01, init_sync=False)
    assert ddp.world_size == 8
    sizes = ddp.bucket_sizes()
    assert len(sizes) > 2 and sum(sizes) == ddp.flat.total
    # reverse registration order: the first bucket (launched first in backward) holds the last parameters
    names = [n for n, p in m.named_parameters() if p.requires_grad]
    first = ddp.buckets[0]
    assert ddp.flat.names[min(first.param_ids)] == names[-1]
    assert ddp.flat.names[max(ddp.buckets[-1].param_ids)] == names[0]
    x = torch.randint(0, 128, (2, 17))
    lo = ddp(x[:, :-1])
    F.cross_entropy(lo.reshape(-1, lo.shape[-1]), x[:, 1:].reshape(-1)).backward()
    assert all(ddp.flat.grad_is_view(i) for i in range(len(ddp.flat.params)))


def test_ddp_buckets_sized_for_xgmi_and_padded():
    """bucket_cap_mb="auto": caps from the xGMI model (>= 6 buckets of overlap, latency
    <= 10 % of a bucket), every bucket boundary a multiple of world_size x 64 elements,
    buckets cover the parameters in reverse registration order without overlap."""
    import torch.nn as nn

    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.flat import xgmi_bucket_caps

    class FakeComm:
        world_size, rank = 8, 0

        def all_reduce(self, t, op="sum"):
            pass

        def broadcast(self, t, src=0):
            pass

    model = nn.Sequential(*[nn.Linear(1000, 1003) for _ in range(12)])
    ddp = DistributedDataParallel(model, comm=FakeComm(), device=torch.device("cpu"), bucket_cap_mb="auto",
                                  init_sync=False)
    grad_bytes = sum(p.numel() for p in model.parameters()) * 4
    first, cap = xgmi_bucket_caps(8, grad_bytes)
    assert ddp.bucket_bytes == (first, cap) and 4 << 20 <= cap <= 64 << 20
    assert len(ddp.buckets) >= 3
    prev_end = 0
    for b in ddp.buckets:
        assert b.start == prev_end or b.start % (8 * 64) == 0
        assert b.end % (8 * 64) == 0, b
        prev_end = b.end
        for i in b.param_ids:
            o, n = ddp.flat.offsets[i], ddp.flat.numels[i]
            assert b.start <= o and o + n <= b.end
    ids = [i for b in ddp.buckets for i in b.param_ids]
    assert ids == list(range(len(ddp.flat.params)))
    assert ddp.flat.names[0] == "11.bias"  # reverse registration order: last layer's grads fill bucket 0


def test_ddp_bucket_caps_from_measured_allreduce_times():
    """bucket_cap_mb="auto" with a calibrated communicator: the caps come from the α/β fit of the
    all-reduce timings the routed communicator measured at wrap, not from the
    assumed xGMI constants -- pinned here with a fixed fake timing table."""
    import torch.nn as nn

    from distributed_training_amd.parallel.comm import Communicator
    from distributed_training_amd.parallel.ddp import DistributedDataParallel
    from distributed_training_amd.parallel.flat import fit_alpha_beta, measured_bucket_caps
    from distributed_training_amd.parallel.routed import MiB, SIZES, RoutedComm

    class Plane(Communicator):
        def __init__(self, name):
            self.name, self.rank, self.world_size, self.device = name, 0, 8, torch.device("cpu")

        def all_reduce(self, t, op="sum", async_op=False):
            return None

        def broadcast(self, t, src=0, async_op=False):
            return None

    # t(S) = 25 us + S / 120 GB/s on RCCL; the IPC plane wins the 1 MiB class only (8 us + S / 60 GB/s)
    alpha, beta = 25e-6, 120e9
    table = {("all_reduce", torch.bfloat16): ["fast", "primary", "primary", "primary"]}
    comm = RoutedComm(Plane("rccl"), Plane("ipc"), table=table)
    for s in SIZES:
        comm.timings[f"all_reduce bfloat16 {s // MiB}MiB"] = (round((alpha + s / beta) * 1e6, 1),
                                                              round((8e-6 + s / 60e9) * 1e6, 1))
    a, b = comm.alpha_beta("all_reduce", torch.bfloat16)
    # the fit runs over the ROUTED times: the 1 MiB point is the IPC plane's
    want = fit_alpha_beta([(s, ((8e-6 + s / 60e9) if i == 0 else (alpha + s / beta))) for i, s in enumerate(SIZES)])
    assert abs(a - want[0]) < 1e-7 and abs(b / want[1] - 1) < 1e-3
    assert fit_alpha_beta([(MiB, 30e-6), (4 * MiB, 60e-6)]) == pytest.approx((20e-6, 3 * MiB / 30e-6))
    assert fit_alpha_beta([(MiB, 30e-6), (4 * MiB, 20e-6)]) is None  # no positive slope: the model

    model = nn.Sequential(*[nn.Linear(1024, 1024) for _ in range(24)])  # 100.7 MB of bf16 gradients
    ddp = DistributedDataParallel(model, comm=comm, device=torch.device("cpu"), bucket_cap_mb="auto",
                                  param_dtype=torch.bfloat16, init_sync=False)
    grad_bytes = sum(p.numel() for p in model.parameters()) * 2
    assert ddp.bucket_bytes == measured_bucket_caps(grad_bytes, a, b)
    assert ddp.bucket_caps_source.startswith("measured")
    first, cap = ddp.bucket_bytes
    # 10 alpha beta ~ 30 MB > grad / 6 ~ 16.8 MB: the overlap rule (>= 6 buckets) sets the cap
    assert cap == int(min(10 * a * b, grad_bytes / 6)) and first == max(MiB, cap // 16)
    # a plain communicator (no timings): the xGMI model
    from distributed_training_amd.parallel.flat import xgmi_bucket_caps

    ddp2 = DistributedDataParallel(model, comm=Plane("rccl"), device=torch.device("cpu"), bucket_cap_mb="auto",
                                   param_dtype=torch.bfloat16, init_sync=False)
    assert ddp2.bucket_bytes == xgmi_bucket_caps(8, grad_bytes) and ddp2.bucket_caps_source.startswith("xgmi")
