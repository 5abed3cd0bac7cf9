"""Single-process multi-GPU replica data parallelism (reference 01.data_parallel.ipynb).

``RandomDataset(32, 1024)`` in batches of 32 (shuffled), ``SampleModel(32, 2)`` wrapped in
``DataParallel`` when more than one device is visible, ``Adam(lr=1e-3)``, ``loss = output.sum()``.
Every replica prints ``Input shape: torch.Size([8, 32])`` on 4 GPUs, and the loop prints
``Input shape: torch.Size([32, 32]), Output shape: torch.Size([32, 2])`` per step (NB01:300-474).

MI355X path: data resident on cuda:0, replicas fed by peer copies, parameters broadcast and
gradients reduced with grouped RCCL calls over xGMI (parallel/dp.py).
``--devices cpu,cpu,cpu,cpu`` runs the same split on CPU (plumbing).
"""
import argparse

import torch

from pytorch_distributed_training_tutorials_amd.data import DeviceDataLoader, DeviceTensorDataset
from pytorch_distributed_training_tutorials_amd.models.toy import SampleModel
from pytorch_distributed_training_tutorials_amd.ops.loss import sum_loss
from pytorch_distributed_training_tutorials_amd.ops.optim import FusedAdam
from pytorch_distributed_training_tutorials_amd.parallel.dp import DataParallel


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--devices", default=None, help="comma list, e.g. 0,1,2,3 or cpu,cpu (default: all GPUs)")
    ap.add_argument("--input_size", type=int, default=32)
    ap.add_argument("--output_size", type=int, default=2)
    ap.add_argument("--data_size", type=int, default=1024)
    ap.add_argument("--batch_size", type=int, default=32)
    ap.add_argument("--quiet", action="store_true", help="do not print per-replica shapes")
    a = ap.parse_args(argv)
    if a.devices:
        devices = [int(d) if d.isdigit() else d for d in a.devices.split(",")]
    else:
        devices = list(range(torch.cuda.device_count())) or ["cpu"]
    d0 = torch.device("cuda", devices[0]) if isinstance(devices[0], int) else torch.device(devices[0])
    data = torch.randn(a.data_size, a.input_size)
    rand_loader = DeviceDataLoader(DeviceTensorDataset(data.to(d0)), batch_size=a.batch_size, shuffle=True)
    model = SampleModel(a.input_size, a.output_size, verbose=not a.quiet).to(d0)
    if len(devices) > 1:
        print(f"Let's use {len(devices)} devices!")
        model = DataParallel(model, device_ids=devices)
    optimizer = FusedAdam(model.parameters(), lr=0.001)
    for data in rand_loader:
        optimizer.zero_grad()
        output = model(data)
        print(f"Input shape: {data.shape}, Output shape: {output.shape}")
        loss = sum_loss(output)  # native reduction; backward is a broadcast view (K7)
        loss.backward()
        optimizer.step()


if __name__ == "__main__":
    main()
