"""Datasets, DistributedSampler-compatible sampling and device-resident loading."""
from .datasets import DeviceTensorDataset, MyTrainDataset, RandomDataset  # noqa: F401
from .loader import DeviceDataLoader  # noqa: F401
from .sampler import DistributedSampler  # noqa: F401
