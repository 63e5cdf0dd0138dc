"""DistributedSampler index parity and device-resident loader batches."""
import pytest
import torch
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler as TorchDS

from distributed_training_amd.data.datasets import DeviceDataLoader, MyTrainDataset, SyntheticTokens
from distributed_training_amd.parallel.sampler import DistributedSampler


@pytest.mark.parametrize("n,ws,shuffle,drop_last", [(2048, 8, True, False), (1000, 3, True, False),
                                                    (10, 4, False, False), (1001, 4, True, True), (5, 8, True, False)])
def test_sampler_matches_torch(n, ws, shuffle, drop_last):
    ds = list(range(n))
    for rank in range(ws):
        for epoch in (0, 3):
            a = TorchDS(ds, num_replicas=ws, rank=rank, shuffle=shuffle, seed=7, drop_last=drop_last)
            b = DistributedSampler(ds, num_replicas=ws, rank=rank, shuffle=shuffle, seed=7, drop_last=drop_last)
            a.set_epoch(epoch)
            b.set_epoch(epoch)
            assert list(a) == list(b)
            assert len(a) == len(b)


def test_dataset_matches_reference_generation():
    torch.manual_seed(123)
    ref = [(torch.rand(20), torch.rand(1)) for _ in range(50)]  # reference src/data_utils.py:10
    torch.manual_seed(123)
    ds = MyTrainDataset(50)
    for i in range(50):
        x, y = ds[i]
        assert torch.equal(x, ref[i][0]) and torch.equal(y, ref[i][1])
    assert len(ds) == 50 and len(ds.data) == 50


def test_device_loader_matches_torch_dataloader():
    ds = MyTrainDataset(203, seed=1)
    for rank in range(2):
        tds = TorchDS(ds, num_replicas=2, rank=rank)
        dds = DistributedSampler(ds, num_replicas=2, rank=rank)
        tl = DataLoader(ds, batch_size=16, shuffle=False, sampler=tds)
        dl = DeviceDataLoader(ds, 16, sampler=dds)
        for ep in range(2):
            tds.set_epoch(ep)
            dds.set_epoch(ep)
            tb = list(tl)
            db = list(dl)
            assert len(tb) == len(db) == len(dl) == len(tl)
            for (x1, y1), (x2, y2) in zip(tb, db):
                assert torch.equal(x1, x2) and torch.equal(y1, y2)


def test_token_loader():
    ds = SyntheticTokens(10, 8, 100, seed=0)
    dl = DeviceDataLoader(ds, 4, sampler=DistributedSampler(ds, num_replicas=1, rank=0, shuffle=False))
    x, y = next(iter(dl))
    assert x.shape == (4, 8) and torch.equal(x[:, 1:], y[:, :-1])
