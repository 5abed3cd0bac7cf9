#!/usr/bin/env python3
"""Repeat tests/test_dp_mp_gpu.py::test_stream_pipeline_one_gpu_matches_single_queue's check in one
process (diagnostic for an intermittent mismatch seen once in round 5): prints one JSON line per
repetition with the worst relative gradient error, and which parameter it is."""
import json
import sys

import torch

sys.path.insert(0, ".")


def main(reps=int(sys.argv[1]) if len(sys.argv) > 1 else 10, channels_last=True):
    from pytorch_distributed_training_tutorials_amd.models.mp_resnet import PipelineParallelResNet50

    dev = torch.device("cuda", 0)
    torch.backends.cudnn.deterministic = True
    for rep in range(reps):
        torch.manual_seed(3)
        a = PipelineParallelResNet50(split_size=4, num_classes=10, dev0=dev, dev1=dev, streams=True)
        b = PipelineParallelResNet50(split_size=4, num_classes=10, dev0=dev, dev1=dev, streams=False)
        b.load_state_dict(a.state_dict())
        x = torch.randn(12, 3, 64, 64, device=dev)
        if channels_last:
            a, b = a.to(memory_format=torch.channels_last), b.to(memory_format=torch.channels_last)
            x = x.contiguous(memory_format=torch.channels_last)
        outs = []
        for m in (a, b):
            m.train()
            y = m(x)
            y.square().mean().backward()
            torch.cuda.synchronize()
            outs.append((y.detach().clone(), [(n, p.grad.detach().clone()) for n, p in m.named_parameters()]))
        yerr = (outs[0][0] - outs[1][0]).abs().max().item()
        errs = [((ga - gb).abs().max() / (gb.abs().max() + 1e-30)).item() for (n, ga), (_, gb) in zip(outs[0][1], outs[1][1])]
        k = max(range(len(errs)), key=lambda j: errs[j])
        print(json.dumps({"rep": rep, "y_err": yerr, "worst": errs[k], "param": outs[0][1][k][0],
                          "n_bad": sum(e > 1e-5 for e in errs)}), flush=True)


if __name__ == "__main__":
    main()
