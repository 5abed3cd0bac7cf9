"""The DDP toy job behind ``ddp_gpus.py`` / ``ddp_gpus_torchrun.py``.

Reference main (ddp_gpus.py:69-93): dataset of 2048 ``(rand(20),
rand(1))`` pairs, DistributedSampler loader, ``Linear(20, 1)``, ``SGD(lr=1e-2)``,
``Trainer.train(max_epochs)``, ``destroy_process_group()``. Same CLI
(``--max_epochs`` 10, ``--batch_size`` 32 per device); extra flags are
additive: ``--engine {auto,fused,autograd}``, ``--model {linear,mlp}``,
``--dataset_size``, ``--lr``, ``--snapshot``/``--save_every``, ``--metrics``.
"""
from __future__ import annotations

import argparse

import torch

from ..data import DeviceDataLoader, DeviceTensorDataset, DistributedSampler
from ..models.toy import ToyMLP, ddp_toy_model
from ..ops.optim import FusedSGD
from ..parallel import env
from ..utils.trainer import Trainer


def parser(description: str = "simple distributed training job") -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=description)
    p.add_argument("--max_epochs", type=int, default=10, help="Total epochs to train the model")
    p.add_argument("--batch_size", type=int, default=32, help="Input batch size on each device")
    p.add_argument("--engine", default="auto", choices=["auto", "fused", "autograd"])
    p.add_argument("--model", default="linear", choices=["linear", "mlp"])
    p.add_argument("--hidden", type=int, default=64)
    p.add_argument("--classes", type=int, default=10)
    p.add_argument("--dataset_size", type=int, default=2048)
    p.add_argument("--lr", type=float, default=1e-2)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--snapshot", default=None, help="snapshot path for save/resume")
    p.add_argument("--save_every", type=int, default=0)
    p.add_argument("--metrics", default=None, help="JSONL metrics file")
    p.add_argument("--no_graph", action="store_true")
    return p


def build_trainer(args, gpu_id: int) -> Trainer:
    dev = env.device()
    torch.manual_seed(args.seed)
    if args.model == "linear":
        ds = DeviceTensorDataset.synthetic_regression(args.dataset_size, 20, 1, device=dev, seed=args.seed)
        model = ddp_toy_model(20, 1)
    else:
        ds = DeviceTensorDataset.synthetic_classification(args.dataset_size, 20, args.classes, device=dev,
                                                          seed=args.seed)
        model = ToyMLP(20, args.hidden, args.classes)
    loader = DeviceDataLoader(ds, batch_size=args.batch_size, sampler=DistributedSampler(ds))
    opt = FusedSGD(model.parameters(), lr=args.lr)
    return Trainer(model, loader, opt, gpu_id, engine=args.engine, graph=not args.no_graph,
                   snapshot_path=args.snapshot, save_every=args.save_every, metrics_path=args.metrics)


def run(args, gpu_id: int) -> Trainer:
    trainer = build_trainer(args, gpu_id)
    trainer.train(args.max_epochs)
    return trainer
