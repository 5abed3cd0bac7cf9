"""Whole-step hipGraph capture for eager training loops.

A ResNet-50 DDP step issues ~600 kernels from Python (autograd, the native
reducer's bucket hooks, MIOpen, the fused optimizer). On MI355X the GPU then
idles wherever the host falls behind: in the round-3 kernel trace of
``benchmarks/resnet_ddp.py`` 1.4 ms of a 19.2 ms step were gaps of 5 us or more
(after the loss, after the optimizer, around MIOpen helper launches;
profiles/r3_resnet_graph.md). Capturing the step once and replaying it removes
every host launch from the loop: one graph launch per step.

What makes a step capturable here (all true of this package's pieces):
  * no host reads inside the step (FusedSGD/FusedAdam keep their step counters on
    the device, BN tickets re-arm in-kernel, DDP's world-1 reducer issues nothing);
  * static inputs: the caller refreshes the tensors the step reads (``x``, ``y``)
    in place before each replay;
  * collectives on the captured streams: the reducer's comm stream joins the
    capture through its ready/done events, and every captured RCCL collective is
    followed by a device completion mark the communicator's watchdog follows
    (:class:`ops.fused_step.WatchedGraph`), so a stalled replay aborts instead of
    hanging;
  * one-time host work (MIOpen exhaustive find, DDP's bucket rebuild after
    iteration 0, optimizer state allocation) happens in the eager warm-up steps,
    which run on a side stream before capture (the torch.cuda.graph recipe).

Reference loop being accelerated: ``Trainer._run_batch`` ddp_gpus.py:34-39 /
the ResNet-50 train loop NB03:969-992.
"""
from __future__ import annotations

import os
from typing import Callable

import torch

from ..ops.fused_step import WatchedGraph

# memset nodes -> fill-kernel nodes before instantiation (csrc/kernels/graph_memset.hip); 0: keep them
_MEMSET_FIX = os.environ.get("PTDT_GRAPH_MEMSET_FIX", "1") != "0"
_MEMSET_NODE_TYPE = 2  # hipGraphNodeTypeMemset


def _detach(out):
    if isinstance(out, torch.Tensor):
        return out.detach()
    if isinstance(out, (tuple, list)):
        return type(out)(_detach(o) for o in out)
    if isinstance(out, dict):
        return {k: _detach(v) for k, v in out.items()}
    return out


class GraphedStep:
    """``step = GraphedStep(fn, device, comm=comm)``; ``out = step()`` replays.

    ``fn`` runs one full training step (zero_grad, forward, backward, optimizer) and
    returns its outputs (e.g. the loss tensor). ``warmup`` eager calls run first on a
    side stream -- they ARE training steps (the trajectory simply starts with them).
    The returned outputs are static tensors overwritten by every replay."""

    def __init__(self, fn: Callable[[], object], device: torch.device, comm=None, warmup: int = 3):
        if device.type != "cuda":
            raise ValueError("GraphedStep needs a GPU device")
        self.fn = fn
        self.device = device
        self.comm = comm
        self._stream = torch.cuda.Stream(device)
        self._stream.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(self._stream):
            for _ in range(max(1, warmup)):
                fn()
        torch.cuda.current_stream(device).wait_stream(self._stream)
        torch.cuda.synchronize(device)
        self.graph = None
        self.captures = 0
        self._capture()
        self.replays = 0
        self._dirty = False

    def _capture(self):
        rc = getattr(self.comm, "handle", None) if self.comm is not None else None
        before = rc.captured if rc is not None else 0
        self.graph = None  # the old graph (and its memory pool) goes first
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g, stream=self._stream, capture_error_mode="thread_local"):
            # detached: a captured loss that keeps its autograd graph alive also keeps every
            # parameter's AccumulateGrad node alive -- nodes created on the capture stream, which
            # later EAGER steps on another stream would then reuse: gradient accumulation and the
            # DDP hooks run on the capture stream while their inputs come from the eager one
            # (cross-stream frees of gradient buffers)
            self.outputs = _detach(self.fn())
        # edit the raw graph before instantiation: MIOpen's hipMemsetAsync calls (atomic
        # weight-gradient solvers) become fill-kernel nodes (profiles/r4_graph_memset.md)
        from .. import native

        raw = g.raw_cuda_graph()
        census = native().graph_node_census(raw)
        self.node_count, self.memset_nodes = int(census[0]), int(census[1 + _MEMSET_NODE_TYPE])
        # [dst, value, elementSize, width, height, pitch] of each captured memset (diagnostics)
        self.memset_params = [list(map(int, p)) for p in native().graph_memset_params(raw)] if self.memset_nodes else []
        self.memsets_replaced = native().graph_replace_memsets(raw) if _MEMSET_FIX else 0
        g.instantiate()
        torch.cuda.synchronize(self.device)
        self.graph = WatchedGraph(g, rc, (rc.captured - before) if rc is not None else 0)
        self.captures += 1

    @property
    def n_collectives(self) -> int:
        return self.graph.n_collectives

    def eager(self):
        """Run the step eagerly. If the instantiated graph still holds memset nodes (the rewrite is
        off, ``PTDT_GRAPH_MEMSET_FIX=0``, or a node could not be rewritten) the next replay
        re-captures first: on ROCm 7 a memset node of an instantiated graph (MIOpen's atomic
        weight-gradient solvers zero their outputs with hipMemsetAsync) stopped zeroing its buffer
        once eager hipMemsetAsync calls had run after the instantiation (profiles/r4_graph_memset.md,
        profiles/r5_graph_memset.md) -- replaying the old graph after eager steps summed weight
        gradients onto stale memory (the round-3 ResNet-50 ``--graph auto`` divergence). With every
        memset node rewritten as a fill kernel there is nothing to re-capture.

        A re-capture runs ``fn``'s Python body once more under capture: its host-side effects
        (DDP forward counters, reducer preparation, logging -- guard those with
        ``torch.cuda.is_current_stream_capturing()``) happen again, and it pays a capture, an
        instantiation and a new memory pool."""
        if self.memset_nodes > self.memsets_replaced:
            self._dirty = True
        return self.fn()

    def __call__(self):
        if self._dirty:
            self._capture()
            self._dirty = False
        self.graph.replay()
        self.replays += 1
        return self.outputs

    def reset(self):
        self.graph.reset()
