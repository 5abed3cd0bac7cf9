#!/usr/bin/env python3
"""ResNet-50 training-loss curves on one fixed synthetic batch: the native step (native DDP
reducer, fused BN kernels, conv+BN statistics fusion, FusedSGD with bf16 weight shadows; eager and
hipGraph-replayed) against stock PyTorch (nn.BatchNorm2d via MIOpen, torch.optim.SGD), same init,
same data, same hyper-parameters as benchmarks/resnet_ddp.py. One JSON line per variant with the
per-step losses -- a numerics check of whole training runs, not a timing.

    python benchmarks/resnet_loss_curve.py [--steps 60] [--batch 128] [--image 224] [--lr 0.1]
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--variants", default="torch,native_eager,native_graph")
    ap.add_argument("--deterministic", action="store_true", help="MIOpen deterministic convolutions")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = not a.deterministic
    torch.backends.cudnn.deterministic = a.deterministic
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel import env
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel

    env.init_process_group("nccl")
    dev = env.device()
    comm = comm_mod.get_default(dev)
    torch.manual_seed(0)
    base = resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.rand(a.batch, 3, a.image, a.image, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev, generator=g)

    for variant in a.variants.split(","):
        if variant == "torch":
            model = resnet50(num_classes=1000, norm_layer=torch.nn.BatchNorm2d).to(dev).to(
                memory_format=torch.channels_last)
            model.load_state_dict(base.state_dict())
            opt = torch.optim.SGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4)

            def step():
                opt.zero_grad()
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = model(x)
                loss = torch.nn.functional.cross_entropy(out.float(), y)
                loss.backward()
                opt.step()
                return loss
        else:
            model = copy.deepcopy(base)
            ddp = DistributedDataParallel(model, device_ids=[dev.index], comm=comm)
            opt = FusedSGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4, bf16_shadow=True)
            graphed = variant == "native_graph"

            def step(ddp=ddp, opt=opt, graphed=graphed):
                ddp.zero_grad()
                with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=not graphed):
                    out = ddp(x)
                loss = cross_entropy(out.float(), y)
                loss.backward()
                opt.step()
                return loss

            if graphed:
                from pytorch_distributed_training_tutorials_amd.utils.graphs import GraphedStep

                step = GraphedStep(step, dev, comm=comm, warmup=3)
        losses = []
        first = 4 if variant == "native_graph" else 1  # GraphedStep ran 3 eager warm-up steps already
        for _ in range(a.steps - first + 1):
            losses.append(round(float(step().detach()), 4))
        torch.cuda.synchronize(dev)
        print(json.dumps({"variant": variant, "steps": a.steps, "batch": a.batch, "image": a.image, "lr": a.lr,
                          "deterministic": a.deterministic, "first_step": first, "losses": losses}), flush=True)
    env.destroy_process_group()


if __name__ == "__main__":
    main()
