"""Two-stage model-parallel ResNet-50 (reference NB03:807-833).

:class:`ModelParallelResNet50` reproduces the reference split exactly:
``seq1 = conv1, bn1, relu, maxpool, layer1, layer2`` on ``dev0``;
``seq2 = layer3, layer4, avgpool`` and ``fc`` on ``dev1``; forward
``seq1(x).to(dev1) -> seq2 -> fc(x.view(B, -1))``. ``seq1``/``seq2`` alias the
base modules like the reference, so ``parameters()`` dedupes (25,557,032) while
``state_dict()`` carries duplicate keys (quirk Q10); :meth:`clean_state_dict`
returns the torchvision-layout dict without the aliases.

On MI355X the activation hop ``[B,512,16,16]`` (62.9 MB fp32 at B=120) is a
``hipMemcpyPeerAsync`` over xGMI issued on the consumer's stream (non-blocking),
~0.4 ms per link at 153 GB/s.

:class:`PipelineParallelResNet50` is the micro-batched extension (GPipe-style
fill/drain with ``split_size`` chunks): stage 0 computes micro-batch i+1 while
stage 1 computes micro-batch i, so the two GPUs overlap instead of idling in
turn (the reference's naive split leaves one GPU idle at all times, §3.4).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .resnet import Bottleneck, ResNet


class ModelParallelResNet50(ResNet):
    def __init__(self, num_classes: int = 1000, dev0="cuda:0", dev1="cuda:1", *args, **kwargs):
        super().__init__(Bottleneck, (3, 4, 6, 3), num_classes=num_classes, *args, **kwargs)
        self.dev0 = torch.device(dev0)
        self.dev1 = torch.device(dev1)
        self.seq1 = nn.Sequential(self.conv1, self.bn1, self.relu, self.maxpool, self.layer1, self.layer2).to(self.dev0)
        self.seq2 = nn.Sequential(self.layer3, self.layer4, self.avgpool).to(self.dev1)
        self.fc.to(self.dev1)

    def forward(self, x):
        x = self.seq2(self.seq1(x.to(self.dev0)).to(self.dev1, non_blocking=True))
        return self.fc(x.view(x.size(0), -1))

    def clean_state_dict(self):
        """state_dict without the ``seq1.*`` / ``seq2.*`` alias duplicates (torchvision layout)."""
        return {k: v for k, v in self.state_dict().items() if not k.startswith(("seq1.", "seq2."))}


class PipelineParallelResNet50(ModelParallelResNet50):
    """Micro-batched two-stage pipeline (the reference tutorial's fill/drain schedule:
    one queue per device). ``streams=True`` runs each stage on its own HIP stream
    instead: stage 0 of micro-batch i+1 and stage 1 of micro-batch i are ordered only by
    one event per micro-batch, and autograd replays each op's backward on its forward's
    stream -- on two GPUs the stages overlap, on one GPU they share the CUs.

    Round 2 saw weight gradients ~7 % apart between this schedule and the single-queue
    one on one device and refused it there. Root cause (benchmarks/pipeline_stream_probe.py,
    profiles/r3_pipeline_stream_probe.md): MIOpen's default convolution weight-gradient
    solvers are not deterministic -- two single-queue runs of the SAME schedule differ by up
    to 9 % on small layer4 gradients. With deterministic algorithms
    (``torch.backends.cudnn.deterministic = True``) the stream schedule matches the
    single-queue one to 6e-6 relative, and it is allowed on one device (tests/test_dp_mp_gpu.py).

    It was NOT race-free by itself: round 5 found the fused BNs' residual-gradient side
    channel (ops/norm.ResidualLink) crossing the stage streams outside autograd's edges
    (23 of 25 repetitions mismatched, tools/stream_pipeline_repeat.py); the link now records
    the stream that produced its stored value -- the sum's stream after a second delivery,
    round 6 -- and the taker waits for it (tests/test_norm.py two-stream delivery tests).
    """

    def __init__(self, split_size: int = 20, *args, streams: bool = False, **kwargs):
        super().__init__(*args, **kwargs)
        self.split_size = split_size
        self.streams = streams
        self._stage_streams = None

    def _forward_single_queue(self, x):
        splits = iter(x.to(self.dev0).split(self.split_size, dim=0))
        s_next = next(splits)
        s_prev = self.seq1(s_next).to(self.dev1, non_blocking=True)
        ret = []
        for s_next in splits:
            # stage 1 on micro-batch i (dev1) while stage 0 runs micro-batch i+1 (dev0): both queues busy
            s_prev = self.seq2(s_prev)
            ret.append(self.fc(s_prev.view(s_prev.size(0), -1)))
            s_prev = self.seq1(s_next).to(self.dev1, non_blocking=True)
        s_prev = self.seq2(s_prev)
        ret.append(self.fc(s_prev.view(s_prev.size(0), -1)))
        return torch.cat(ret)

    def forward(self, x):
        if not (self.streams and x.is_cuda and self.dev0.type == "cuda" and self.dev1.type == "cuda"):
            return self._forward_single_queue(x)
        if self._stage_streams is None:
            self._stage_streams = (torch.cuda.Stream(self.dev0), torch.cuda.Stream(self.dev1))
        s0, s1 = self._stage_streams
        cur0, cur1 = torch.cuda.current_stream(self.dev0), torch.cuda.current_stream(self.dev1)
        x = x.to(self.dev0)
        s0.wait_stream(cur0)  # the input and the parameters as the caller's queue left them
        s1.wait_stream(cur1)
        outs = []
        for chunk in x.split(self.split_size, dim=0):
            with torch.cuda.stream(s0):
                a = self.seq1(chunk)
                chunk.record_stream(s0)
            ready = torch.cuda.Event()
            ready.record(s0)
            with torch.cuda.device(self.dev1), torch.cuda.stream(s1):
                s1.wait_event(ready)
                b = a.to(self.dev1, non_blocking=True)  # the hop, on the consumer's queue
                a.record_stream(s1)
                b = self.seq2(b)
                outs.append(self.fc(b.view(b.size(0), -1)))
        cur1.wait_stream(s1)
        for o in outs:
            o.record_stream(cur1)
        return torch.cat(outs)
