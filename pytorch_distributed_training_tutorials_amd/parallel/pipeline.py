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

Wire protocol: EVERY activation / gradient message is preceded by a fixed
88-byte header ``int64[11] = [dtype, ndim, n_micro, d0..d7]`` on the same peer
pair, so the receiver sizes each buffer from what was actually sent, and
learns the step's micro-batch count from stage 0 -- a partial last batch
(20 -> 8 rows) or an uneven micro-batch split (18 rows / 4 = 5,5,5,3; 6 rows /
4 = 2,2,2) needs no configuration and cannot desynchronise the stages. The last
stage slices its targets by the row counts it actually receives.

Overlap (GPU): sends and receives run on a dedicated P2P HIP stream. A send
waits (stream event) for the compute stream that produced the tensor and the
host returns immediately, so stage ``s`` computes micro-batch ``i+1`` while
micro-batch ``i`` is on the link; a receive blocks the host only on the
88-byte header (side-stream event), and the compute stream waits for the
payload with a stream dependency, never a device-wide sync.

Micro-batch losses are weighted by their row share (``rows_i / rows``), so a
mean-reduced loss over an uneven split equals the full-batch loss.
"""
from __future__ import annotations

import torch
import torch.nn as nn

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3, torch.int64: 4, torch.int32: 5}
_DT_INV = {v: k for k, v in _DT.items()}
_HDR = 11  # [dtype, ndim, n_micro, d0..d7]
_MAXDIM = _HDR - 3


def _header(t: torch.Tensor, n_micro: int) -> torch.Tensor:
    if t.dim() > _MAXDIM:
        raise ValueError(f"PipelineStage: tensors of rank <= {_MAXDIM} only (got {t.dim()})")
    if t.dtype not in _DT:
        raise ValueError(f"PipelineStage: unsupported dtype {t.dtype}")
    return torch.tensor([_DT[t.dtype], t.dim(), n_micro, *t.shape] + [0] * (_MAXDIM - t.dim()), dtype=torch.int64)


def _parse(h):
    return _DT_INV[h[0]], h[3:3 + h[1]], h[2]


class PipelineStage:
    """One pipeline stage per rank. ``loss_reduction`` says how ``loss_fn`` reduces
    over rows ("mean": micro-batch losses are weighted by their row share; "sum":
    added as they are). ``overlap=False`` runs the P2P on the compute stream."""

    def __init__(self, module: nn.Module, comm, stage: int | None = None, num_stages: int | None = None,
                 loss_fn=None, micro_batches: int = 1, device=None, loss_reduction: str = "mean",
                 overlap: bool = True):
        if loss_reduction not in ("mean", "sum"):
            raise ValueError("loss_reduction must be 'mean' or 'sum'")
        self.module = module
        self.comm = comm
        self.stage = comm.rank if stage is None else stage
        self.num_stages = comm.world if num_stages is None else num_stages
        self.loss_fn = loss_fn
        self.micro_batches = micro_batches
        self.loss_reduction = loss_reduction
        self.device = torch.device(device) if device is not None else next(module.parameters()).device
        self.first = self.stage == 0
        self.last = self.stage == self.num_stages - 1
        gpu = self.device.type == "cuda" and getattr(comm, "native", False)
        self._side = torch.cuda.Stream(self.device) if (gpu and overlap) else None
        self.messages = 0  # payload messages sent + received (tests / tracing)

    # ---------------------------------------------------------------- p2p helpers
    def _send(self, t: torch.Tensor, peer: int, n_micro: int = 0):
        t = t.detach().contiguous()
        hdr = _header(t, n_micro)
        self.messages += 1
        if t.device.type != "cuda":
            self.comm.send(hdr, peer)
            self.comm.send(t, peer)
            return
        if self._side is None:
            self.comm.send(hdr.to(t.device), peer)
            self.comm.send(t, peer)
            return
        cur = torch.cuda.current_stream(self.device)
        self._side.wait_stream(cur)  # the payload is produced on the compute stream
        with torch.cuda.stream(self._side):
            h = hdr.pin_memory().to(self.device, non_blocking=True)
            self.comm.send(h, peer)
            self.comm.send(t, peer)
        # the caching allocator must not hand these blocks to the compute stream before the send read them
        t.record_stream(self._side)
        h.record_stream(self._side)

    def _recv(self, peer: int):
        """-> (tensor, n_micro announced by the sender)."""
        self.messages += 1
        if self.device.type != "cuda":
            hdr = torch.zeros(_HDR, dtype=torch.int64)
            self.comm.recv(hdr, peer)
            dt, shape, nm = _parse(hdr.tolist())
            buf = torch.empty(shape, dtype=dt)
            self.comm.recv(buf, peer)
            return buf, nm
        stream = self._side or torch.cuda.current_stream(self.device)
        with torch.cuda.stream(stream):
            hd = torch.empty(_HDR, dtype=torch.int64, device=self.device)
            self.comm.recv(hd, peer)
            hh = torch.empty(_HDR, dtype=torch.int64, pin_memory=True)
            hh.copy_(hd, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        ev.synchronize()  # host waits for the 88-byte header only
        dt, shape, nm = _parse(hh.tolist())
        with torch.cuda.stream(stream):
            buf = torch.empty(shape, dtype=dt, device=self.device)
            self.comm.recv(buf, peer)
        if self._side is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._side)
            buf.record_stream(torch.cuda.current_stream(self.device))
        return buf, nm

    def synchronize(self):
        """Wait for every P2P this stage issued (end of step / before reading results)."""
        if self._side is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._side)

    # ---------------------------------------------------------------- schedule
    def train_step(self, x: torch.Tensor | None = None, target: torch.Tensor | None = None):
        """One GPipe step. Stage 0 passes ``x``, the last stage ``target``; returns the
        loss on the last stage (None elsewhere). Gradients accumulate in
        ``module``'s parameters (call the optimizer afterwards). Any batch size
        works, including a partial last batch and splits that are not a multiple of
        ``micro_batches``; no stage is told the batch size."""
        xs = list(x.chunk(self.micro_batches)) if self.first else None
        n_mb = len(xs) if xs is not None else None  # later stages: from the first header
        rows_total = target.shape[0] if self.last else None
        inputs, outputs, losses = [], [], []
        row = 0
        i = 0
        while n_mb is None or i < n_mb:  # fill: all forwards
            if self.first:
                inp = xs[i].to(self.device, non_blocking=True)
            else:
                inp, nm = self._recv(self.stage - 1)
                inp.requires_grad_(True)
                n_mb = nm if n_mb is None else n_mb
            out = self.module(inp)
            inputs.append(inp)
            if self.last:
                r = out.shape[0]
                t = target[row:row + r].to(self.device, non_blocking=True)
                row += r
                loss = self.loss_fn(out, t)
                if self.loss_reduction == "mean":
                    loss = loss * (r / rows_total)
                losses.append(loss)
                outputs.append(loss)
            else:
                self._send(out, self.stage + 1, n_mb)
                outputs.append(out)
            i += 1
        if self.last and row != rows_total:
            raise RuntimeError(f"PipelineStage: received {row} rows for a target of {rows_total}")
        for i in reversed(range(len(outputs))):  # drain: backwards in reverse
            if self.last:
                outputs[i].backward()
            else:
                g, _ = self._recv(self.stage + 1)
                outputs[i].backward(g)
            if not self.first:
                gi = inputs[i].grad
                self._send(gi if gi is not None else torch.zeros_like(inputs[i]), self.stage - 1)
        self.synchronize()
        if self.last:
            return torch.stack([l.detach() for l in losses]).sum()
        return None

    @torch.no_grad()
    def forward(self, x: torch.Tensor | None = None) -> torch.Tensor | None:
        """Inference through the pipeline; returns the output on the last stage."""
        inp = x.to(self.device) if self.first else self._recv(self.stage - 1)[0]
        out = self.module(inp)
        if not self.last:
            self._send(out, self.stage + 1, 1)
            self.synchronize()
            return None
        return out
