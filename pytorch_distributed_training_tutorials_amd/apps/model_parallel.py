"""Model-parallel demos and the MP-vs-single-GPU ResNet-50 benchmark
(reference 03.model_parallel.ipynb).

* :func:`toy_step` -- ``ToyModel`` (Linear(10000,10)+ReLU on dev0, Linear(10,5) on
  dev1), one MSE/SGD step (NB03:440-542).
* :func:`train` -- the reference's ``train(model)``: 3 batches of
  ``[120, 3, 128, 128]`` with one-hot MSE targets and SGD(lr=1e-3)
  (NB03:969-992). Inputs and one-hot labels are generated on the GPU
  (Philox + one-hot kernels) instead of CPU randn + pageable H2D copies
  (SURVEY K18/K19, M13).
* :func:`benchmark` -- ``timeit.repeat(train, number=1, repeat=10)`` for the
  2-stage split, the micro-batched pipeline and the single-GPU model, with
  ``torch.cuda.synchronize()`` inside the timed statement (the reference times
  without one, quirk Q8) and the bar chart saved to a file (quirk Q9).
"""
from __future__ import annotations

import json
import timeit

import numpy as np
import torch
import torch.nn as nn

from .._ext import native
from ..models.mp_resnet import ModelParallelResNet50, PipelineParallelResNet50
from ..models.resnet import resnet50
from ..models.toy import ToyModel, model_size
from ..ops.loss import mse_loss
from ..ops.optim import FusedSGD

NUM_CLASSES = 1000
NUM_BATCHES = 3
BATCH_SIZE = 120
IMAGE_W = IMAGE_H = 128


def toy_step(dev0="cuda:0", dev1="cuda:1", verbose=True):
    model = ToyModel(dev0, dev1)
    if verbose:
        print(f"net1 on {model.net1.weight.device}, net2 on {model.net2.weight.device}; "
              f"{model_size(model)} parameters")
    loss_fn = nn.MSELoss()
    opt = FusedSGD(model.parameters(), lr=0.001)
    opt.zero_grad()
    outputs = model(torch.randn(20, 10000))
    labels = torch.randn(20, 5).to(outputs.device)
    loss = loss_fn(outputs, labels)
    loss.backward()
    opt.step()
    return float(loss.detach())


def _batch(dev, seed: int, one_hot_idx):
    x = torch.empty(BATCH_SIZE, 3, IMAGE_W, IMAGE_H, device=dev)
    if dev.type == "cuda":
        native().philox_(x, seed, 0, 1)
        labels = native().one_hot(one_hot_idx.to(dev), NUM_CLASSES)
    else:
        x.normal_(generator=torch.Generator().manual_seed(seed))
        labels = torch.zeros(BATCH_SIZE, NUM_CLASSES).scatter_(1, one_hot_idx.view(-1, 1), 1)
    return x, labels


def train(model, in_dev=None, sync=True, seed: int = 0):
    """Reference ``train(model)`` (NB03:974-992)."""
    model.train(True)
    opt = FusedSGD(model.parameters(), lr=0.001)
    g = torch.Generator().manual_seed(seed)
    one_hot_indices = torch.randint(0, NUM_CLASSES, (BATCH_SIZE,), generator=g)
    in_dev = in_dev or next(model.parameters()).device
    for i in range(NUM_BATCHES):
        inputs, labels = _batch(in_dev, seed * 1000 + i, one_hot_indices)
        opt.zero_grad()
        outputs = model(inputs)
        labels = labels.to(outputs.device)
        mse_loss(outputs, labels).backward()
        opt.step()
    if sync and torch.cuda.is_available():
        torch.cuda.synchronize()


def benchmark(repeat: int = 10, devs=("cuda:0", "cuda:1"), split_sizes=(20,), channels_last: bool = False,
              fig: str | None = "mp_vs_single.png", json_out: str | None = None):
    def cl(m):
        return m.to(memory_format=torch.channels_last) if channels_last else m

    results = {}
    setups = {"Model Parallel": lambda: cl(ModelParallelResNet50(NUM_CLASSES, devs[0], devs[1])),
              "Single GPU": lambda: cl(resnet50(num_classes=NUM_CLASSES).to(devs[0]))}
    for ss in split_sizes:
        setups[f"Pipeline split={ss}"] = (lambda ss=ss: cl(PipelineParallelResNet50(ss, NUM_CLASSES, devs[0], devs[1])))
        if devs[0] != devs[1]:  # stage streams: two GPUs only
            setups[f"Pipeline split={ss} stage streams"] = (
                lambda ss=ss: cl(PipelineParallelResNet50(ss, NUM_CLASSES, devs[0], devs[1], streams=True)))
    for name, mk in setups.items():
        model = mk()
        in_dev = torch.device(devs[0])
        print(f"[mp bench] {name}: warm-up (MIOpen solver search, allocator)", flush=True)
        train(model, in_dev)  # warm-up (MIOpen solver search, allocator)
        times = timeit.repeat(lambda: train(model, in_dev), number=1, repeat=repeat)
        results[name] = {"mean_s": float(np.mean(times)), "std_s": float(np.std(times)),
                         "img_per_s": NUM_BATCHES * BATCH_SIZE / float(np.mean(times))}
        del model
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
    if fig:
        plot([r["mean_s"] for r in results.values()], [r["std_s"] for r in results.values()], list(results), fig)
    if json_out:
        with open(json_out, "w") as f:
            json.dump(results, f, indent=1)
    return results


def plot(means, stds, labels, fig_name):
    """Bar chart "ResNet50 Execution Time (Second)" (reference NB03:1047-1055), saved to ``fig_name``."""
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    fig, ax = plt.subplots()
    ax.bar(np.arange(len(means)), means, yerr=stds, align="center", alpha=0.5, ecolor="red", capsize=10, width=0.6)
    ax.set_ylabel("ResNet50 Execution Time (Second)")
    ax.set_xticks(np.arange(len(means)))
    ax.set_xticklabels(labels, rotation=10)
    ax.yaxis.grid(True)
    plt.tight_layout()
    plt.savefig(fig_name)
    plt.close(fig)
