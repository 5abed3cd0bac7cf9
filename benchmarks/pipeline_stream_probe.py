#!/usr/bin/env python3
"""Diagnose the same-device stage-stream pipeline: stream schedule vs single-queue schedule,
max gradient difference (run with and without PYTORCH_NO_HIP_MEMORY_CACHING=1)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_training_tutorials_amd.models.mp_resnet import PipelineParallelResNet50  # noqa: E402

dev = "cuda:0"
torch.manual_seed(3)
a = PipelineParallelResNet50(split_size=4, num_classes=10, dev0=dev, dev1=dev, streams="force")
b = PipelineParallelResNet50(split_size=4, num_classes=10, dev0=dev, dev1=dev, streams=False)
b.load_state_dict(a.state_dict())
x = torch.randn(12, 3, 64, 64, device=dev)
res = []
for m in (a, b):
    m.train()
    y = m(x)
    y.square().mean().backward()
    torch.cuda.synchronize()
    res.append((y.detach().clone(), [p.grad.detach().clone() for p in m.parameters()]))
dy = (res[0][0] - res[1][0]).abs().max().item()
dg = max((ga - gb).abs().max().item() / (gb.abs().max().item() + 1e-12) for ga, gb in zip(res[0][1], res[1][1]))
print({"caching": os.environ.get("PYTORCH_NO_HIP_MEMORY_CACHING", "on"), "max_out_diff": dy, "max_rel_grad_diff": dg},
      flush=True)
