"""Model parallelism across ranks: stage-to-stage activations over RCCL send/recv.

Reference: naive in-process model parallelism (``ToyModel`` NB03:440-450,
``ModelParallelResNet50`` NB03:807-833): one process
drives two GPUs and moves activations with ``.to("cuda:1")``. Those in-process
forms live in ``models/toy.py`` / ``models/mp_resnet.py`` (peer copies over
xGMI). This module is the multi-process variant the north star asks for --
"the model-parallel stage split uses RCCL send/recv between two ranks" -- with
one process per GPU, each owning one stage:

* forward: stage ``s`` receives its input activation from rank ``s-1``
  (``ncclRecv``), runs its module, sends the output to rank ``s+1``
  (``ncclSend``); the last stage computes the loss;
* backward: the last stage back-propagates and sends d(input) to ``s-1``;
  middle stages receive d(output), back-propagate, send d(input);
* ``micro_batches > 1`` gives the GPipe fill/drain schedule (all forwards, then
  all backwards in reverse), so stage ``s`` works on micro-batch ``i`` while
  stage ``s+1`` works on ``i-1``; ``micro_batches == 1`` is the reference's
  naive, fully serialised split.
Activation shapes/dtypes travel in a small fixed-size header the first time a
(micro-batch, direction) shape is seen, so stages need no shape configuration.
"""
from __future__ import annotations

import torch
import torch.nn as nn

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3}
_DT_INV = {v: k for k, v in _DT.items()}
_HDR = 10  # [dtype, ndim, d0..d7]


class PipelineStage:
    def __init__(self, module: nn.Module, comm, stage: int | None = None, num_stages: int | None = None,
                 loss_fn=None, micro_batches: int = 1, device=None):
        self.module = module
        self.comm = comm
        self.stage = comm.rank if stage is None else stage
        self.num_stages = comm.world if num_stages is None else num_stages
        self.loss_fn = loss_fn
        self.micro_batches = micro_batches
        self.device = device or next(module.parameters()).device
        self.first = self.stage == 0
        self.last = self.stage == self.num_stages - 1
        self._shapes = {}

    # ---------------------------------------------------------------- p2p helpers
    def _send(self, t: torch.Tensor, peer: int, key):
        t = t.contiguous()
        if self._shapes.get(("s", key)) != (t.dtype, tuple(t.shape)):
            hdr = torch.zeros(_HDR, dtype=torch.int64, device=t.device)
            hdr[0], hdr[1] = _DT[t.dtype], t.dim()
            hdr[2:2 + t.dim()] = torch.tensor(t.shape, dtype=torch.int64)
            self.comm.send(hdr, peer)
            self._shapes[("s", key)] = (t.dtype, tuple(t.shape))
        self.comm.send(t, peer)

    def _recv(self, peer: int, key) -> torch.Tensor:
        meta = self._shapes.get(("r", key))
        if meta is None:
            hdr = torch.zeros(_HDR, dtype=torch.int64, device=self.device)
            self.comm.recv(hdr, peer)
            h = hdr.tolist()
            meta = (_DT_INV[h[0]], tuple(h[2:2 + h[1]]))
            self._shapes[("r", key)] = meta
        buf = torch.empty(meta[1], dtype=meta[0], device=self.device)
        self.comm.recv(buf, peer)
        return buf

    # ---------------------------------------------------------------- schedule
    def train_step(self, x: torch.Tensor | None = None, target: torch.Tensor | None = None):
        """One GPipe step. Stage 0 passes ``x``, the last stage ``target``; returns the
        mean loss on the last stage (None elsewhere). Gradients accumulate in
        ``module``'s parameters (call the optimizer afterwards)."""
        m = self.micro_batches
        xs = list(x.chunk(m)) if (self.first and x is not None) else [None] * m
        ts = list(target.chunk(m)) if (self.last and target is not None) else [None] * m
        inputs, outputs, losses = [], [], []
        for i in range(m):  # fill: all forwards
            if self.first:
                inp = xs[i].to(self.device, non_blocking=True)
            else:
                inp = self._recv(self.stage - 1, ("act", i)).requires_grad_(True)
            out = self.module(inp)
            inputs.append(inp)
            if self.last:
                loss = self.loss_fn(out, ts[i].to(self.device, non_blocking=True)) / m
                losses.append(loss)
                outputs.append(loss)
            else:
                self._send(out.detach(), self.stage + 1, ("act", i))
                outputs.append(out)
        for i in reversed(range(m)):  # drain: backwards in reverse
            if self.last:
                outputs[i].backward()
            else:
                g = self._recv(self.stage + 1, ("grad", i))
                outputs[i].backward(g)
            if not self.first:
                self._send(inputs[i].grad, self.stage - 1, ("grad", i))
        if self.last:
            return torch.stack([l.detach() for l in losses]).sum()
        return None

    @torch.no_grad()
    def forward(self, x: torch.Tensor | None = None) -> torch.Tensor | None:
        """Inference through the pipeline; returns the output on the last stage."""
        inp = x.to(self.device) if self.first else self._recv(self.stage - 1, ("fwd",))
        out = self.module(inp)
        if not self.last:
            self._send(out, self.stage + 1, ("fwd",))
            return None
        return out
