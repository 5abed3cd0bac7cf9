"""DistributedSampler parity (bit-identical to torch) and the device sampler's host model."""
import numpy as np
import pytest
import torch
from torch.utils.data.distributed import DistributedSampler as TorchSampler

from pytorch_distributed_training_tutorials_amd.data.device_sampler import reference_indices
from pytorch_distributed_training_tutorials_amd.data.loader import DeviceDataLoader
from pytorch_distributed_training_tutorials_amd.data.datasets import DeviceTensorDataset, MyTrainDataset
from pytorch_distributed_training_tutorials_amd.data.sampler import DistributedSampler


@pytest.mark.parametrize("n", [2048, 1000, 7, 5])
@pytest.mark.parametrize("w", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("drop_last", [False, True])
@pytest.mark.parametrize("shuffle", [True, False])
def test_distributed_sampler_bit_identical(n, w, drop_last, shuffle):
    ds = list(range(n))
    for r in range(w):
        ours = DistributedSampler(ds, num_replicas=w, rank=r, shuffle=shuffle, seed=0, drop_last=drop_last)
        ref = TorchSampler(ds, num_replicas=w, rank=r, shuffle=shuffle, seed=0, drop_last=drop_last)
        for e in (0, 1, 5):
            ours.set_epoch(e)
            ref.set_epoch(e)
            assert list(ours) == list(ref)
            assert len(ours) == len(ref)


def test_steps_per_epoch_match_reference_recordings():
    """NB02:231-272: 2048 samples, batch 32 -> Steps 64 @ W=1, 16 @ W=4."""
    ds = DeviceTensorDataset.synthetic_regression(2048)
    for w, steps in ((1, 64), (2, 32), (4, 16), (8, 8)):
        dl = DeviceDataLoader(ds, batch_size=32, sampler=DistributedSampler(ds, w, 0))
        assert len(dl) == steps


def test_device_loader_cpu_batches_follow_sampler():
    ds = DeviceTensorDataset.synthetic_regression(100, 20, 1)
    s = DistributedSampler(ds, 3, 1, seed=4)
    dl = DeviceDataLoader(ds, batch_size=16, sampler=s)
    dl.set_epoch(2)
    idx = list(s)
    got = torch.cat([x for x, _ in dl])
    torch.testing.assert_close(got, ds.tensors[0][torch.tensor(idx)])
    assert [b for _, b in dl.batches()] == [16, 16, 2]


@pytest.mark.parametrize("n,w", [(2048, 1), (2048, 8), (1000, 3), (5, 8), (4097, 4), (1, 1)])
def test_device_sampler_model_partitions_dataset(n, w):
    for e in (0, 1, 9):
        shards = [reference_indices(n, w, r, e, seed=11) for r in range(w)]
        cat = np.concatenate(shards)
        assert len(cat) == -(-n // w) * w
        assert set(cat.tolist()) == set(range(n))  # every sample seen; padding only repeats
        if n % w == 0:
            assert sorted(cat.tolist()) == list(range(n))
    a = reference_indices(n, w, 0, 0, seed=11)
    b = reference_indices(n, w, 0, 1, seed=11)
    if n > 8:
        assert not np.array_equal(a, b)  # epochs reshuffle


def test_mytraindataset_shapes_and_seeding():
    a = MyTrainDataset(2048)
    b = MyTrainDataset(2048)
    x, y = a[0]
    assert x.shape == (20,) and y.shape == (1,) and len(a) == 2048
    torch.testing.assert_close(a.x, b.x)
    c = MyTrainDataset(16, rank=1, per_rank_seed=True)
    assert not torch.equal(c.x, MyTrainDataset(16, rank=0, per_rank_seed=True).x)
