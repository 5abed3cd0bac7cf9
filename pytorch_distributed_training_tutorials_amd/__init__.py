"""MI355X-native distributed-training harness with the capabilities of
duoan/pytorch_distributed_training_tutorials (DataParallel, DistributedDataParallel,
naive model parallel), built on PyTorch-ROCm + hand-written gfx950 HIP kernels +
a native RCCL communicator / DDP reducer.

Subpackages: ``ops`` (native kernels with autograd), ``parallel`` (process groups,
communicator, DDP, DP, pipeline/model parallel, placement, launcher), ``models``,
``data``, ``utils`` (trainer, checkpoint, metrics, tracing, faults).
"""
__version__ = "0.1.0"

from ._ext import has_native, native  # noqa: F401
