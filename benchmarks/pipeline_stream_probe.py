#!/usr/bin/env python3
"""Diagnose the same-device stage-stream pipeline (models/mp_resnet.py).

Compares the training step of ``PipelineParallelResNet50(streams=True)`` (stage 0 and
stage 1 on two HIP streams of ONE device) with the single-queue schedule, per parameter,
under several conditions, one JSON line each:

* ``sq_vs_sq``    -- two single-queue runs from the same state: the run-to-run noise floor
                     (non-deterministic reductions in the library kernels);
* ``streams``     -- stream schedule vs single queue (the round-2 finding: ~7 %);
* ``streams_det`` -- the same with ``torch.backends.cudnn.deterministic = True``;
* ``streams_cl``  -- channels_last input (native NHWC BN / pool kernels instead of MIOpen BN).

Error metric per parameter: max |g_a - g_b| / max |g_b|; ``worst`` lists the 3 largest.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_training_tutorials_amd.models.mp_resnet import PipelineParallelResNet50  # noqa: E402

dev = "cuda:0"


def step(m, x):
    m.train()
    for p in m.parameters():
        p.grad = None
    y = m(x)
    y.square().mean().backward()
    torch.cuda.synchronize()
    return y.detach().clone(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}


def compare(tag, ra, rb):
    dy = (ra[0] - rb[0]).abs().max().item()
    errs = []
    for n, gb in rb[1].items():
        ga = ra[1][n]
        errs.append(((ga - gb).abs().max().item() / (gb.abs().max().item() + 1e-30), n, gb.abs().max().item()))
    errs.sort(reverse=True)
    print(json.dumps({"case": tag, "max_out_diff": dy, "max_rel_grad_diff": errs[0][0],
                      "worst": [{"param": n, "rel": round(e, 6), "grad_absmax": g} for e, n, g in errs[:3]]}),
          flush=True)


def build(streams, seed=3):
    torch.manual_seed(seed)
    return PipelineParallelResNet50(split_size=4, num_classes=10, dev0=dev, dev1=dev, streams=streams)


def main():
    torch.manual_seed(3)
    x = torch.randn(12, 3, 64, 64, device=dev)
    ref = build(False)
    state = {k: v.clone() for k, v in ref.state_dict().items()}

    def fresh(streams):
        m = build(streams)
        m.load_state_dict(state)
        return m

    base = step(fresh(False), x)
    compare("sq_vs_sq", step(fresh(False), x), base)
    compare("streams", step(fresh(True), x), base)
    torch.backends.cudnn.deterministic = True
    base_det = step(fresh(False), x)
    compare("sq_vs_sq_det", step(fresh(False), x), base_det)
    compare("streams_det", step(fresh(True), x), base_det)
    torch.backends.cudnn.deterministic = False
    xcl = x.contiguous(memory_format=torch.channels_last)

    def fresh_cl(streams):
        return fresh(streams).to(memory_format=torch.channels_last)

    base_cl = step(fresh_cl(False), xcl)
    compare("sq_vs_sq_cl", step(fresh_cl(False), xcl), base_cl)
    compare("streams_cl", step(fresh_cl(True), xcl), base_cl)


if __name__ == "__main__":
    main()
