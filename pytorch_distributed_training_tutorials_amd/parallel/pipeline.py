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

Wire protocol (one host round trip per step per stage, none per micro-batch):
at the start of a step stage ``s`` sends stage ``s+1`` ONE step header --
``int64[3 + 7 + 64] = [dtype, ndim, n_micro, trailing dims d1..d7, rows_0 ..
rows_{n_micro-1}]``, written after its first micro-batch forward (the first point
where the output's dtype and trailing dims are known). The receiver reads it on
the host once, and from then on sizes every payload of the step from it: forward
activations are ``[rows_i, *trailing]``, and backward gradients carry no header
at all (a gradient has the shape and dtype of the activation it belongs to, which
both ends already hold). A partial last batch (20 -> 8 rows) or an uneven
micro-batch split (18 rows / 4 = 5,5,5,3; 6 rows / 4 = 2,2,2) needs no
configuration: stage 0's chunking travels down the pipeline in the headers. The
last stage slices its targets by the row counts it receives.

Restriction: a stage must keep the row count (every stage maps a micro-batch of
``r`` rows to ``r`` rows) and one dtype / trailing shape for all micro-batches of a
step -- the step header is written once, after micro-batch 0. A violation found at
micro-batch 0 raises before anything is sent. One found later (micro-batch i > 0,
after the header went out), or a last stage whose rows do not add up to its
target, still completes the step's wire protocol -- zero payloads of the advertised
shape forward, zero gradients backward -- and raises at the end of the step, so no
peer is left blocked mid-step on this rank's messages.

Overlap (GPU): sends and receives run on a dedicated P2P HIP stream. A send
waits (stream event) for the compute stream that produced the tensor and the
host returns immediately, so stage ``s`` computes micro-batch ``i+1`` while
micro-batch ``i`` is on the link; payload receives are pure stream dependencies
(the compute stream waits for the P2P stream), so after the step header the host
never waits on a peer.

Micro-batch losses are weighted by their row share (``rows_i / rows``), so a
mean-reduced loss over an uneven split equals the full-batch loss.
"""
from __future__ import annotations

import torch
import torch.nn as nn

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3, torch.int64: 4, torch.int32: 5}
_DT_INV = {v: k for k, v in _DT.items()}
_MAXDIM = 8   # tensor rank (leading row dim + 7 trailing)
_MAXMB = 64   # micro-batches per step
_HDR = 3 + (_MAXDIM - 1) + _MAXMB  # [dtype, ndim, n_micro, d1..d7, rows_0..rows_63]


def _step_header(t: torch.Tensor, rows) -> torch.Tensor:
    """The step header of a link: ``t`` is micro-batch 0's payload, ``rows`` every micro-batch's rows."""
    if t.dim() < 1 or t.dim() > _MAXDIM:
        raise ValueError(f"PipelineStage: activations of rank 1..{_MAXDIM} only (got {t.dim()})")
    if t.dtype not in _DT:
        raise ValueError(f"PipelineStage: unsupported dtype {t.dtype}")
    if not 1 <= len(rows) <= _MAXMB:
        raise ValueError(f"PipelineStage: 1..{_MAXMB} micro-batches per step (got {len(rows)})")
    trail = list(t.shape[1:])
    return torch.tensor([_DT[t.dtype], t.dim(), len(rows), *trail, *([0] * (_MAXDIM - 1 - len(trail))),
                         *rows, *([0] * (_MAXMB - len(rows)))], dtype=torch.int64)


def _parse(h):
    """-> (dtype, trailing dims, per-micro-batch rows)."""
    nd, nm = h[1], h[2]
    return _DT_INV[h[0]], tuple(h[3:3 + nd - 1]), list(h[3 + _MAXDIM - 1:3 + _MAXDIM - 1 + nm])


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
        self.headers = 0   # step headers received: one per step on every stage but the first

    # ---------------------------------------------------------------- p2p helpers
    def _send_header(self, hdr: torch.Tensor, peer: int):
        if self.device.type != "cuda":
            self.comm.send(hdr, peer)
            return
        if self._side is None:
            self.comm.send(hdr.to(self.device), peer)
            return
        with torch.cuda.stream(self._side):
            h = hdr.pin_memory().to(self.device, non_blocking=True)
            self.comm.send(h, peer)
        h.record_stream(self._side)

    def _recv_header(self, peer: int):
        """The step header from ``peer``: the one host wait of a step on this link."""
        self.headers += 1
        if self.device.type != "cuda":
            hdr = torch.zeros(_HDR, dtype=torch.int64)
            self.comm.recv(hdr, peer)
            return _parse(hdr.tolist())
        stream = self._side or torch.cuda.current_stream(self.device)
        with torch.cuda.stream(stream):
            hd = torch.empty(_HDR, dtype=torch.int64, device=self.device)
            self.comm.recv(hd, peer)
            hh = torch.empty(_HDR, dtype=torch.int64, pin_memory=True)
            hh.copy_(hd, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        ev.synchronize()
        return _parse(hh.tolist())

    def _send(self, t: torch.Tensor, peer: int):
        """A payload (no header): the receiver knows its shape from the step header / its own tensors."""
        t = t.detach().contiguous()
        self.messages += 1
        if t.device.type != "cuda" or self._side is None:
            self.comm.send(t, peer)
            return
        cur = torch.cuda.current_stream(self.device)
        self._side.wait_stream(cur)  # the payload is produced on the compute stream
        with torch.cuda.stream(self._side):
            self.comm.send(t, peer)
        # the caching allocator must not hand the block to the compute stream before the send read it
        t.record_stream(self._side)

    def _recv(self, shape, dtype, peer: int) -> torch.Tensor:
        """A payload of known shape: on GPU a stream dependency only (no host wait)."""
        self.messages += 1
        if self.device.type != "cuda":
            buf = torch.empty(shape, dtype=dtype)
            self.comm.recv(buf, peer)
            return buf
        if self._side is None:
            buf = torch.empty(shape, dtype=dtype, device=self.device)
            self.comm.recv(buf, peer)
            return buf
        with torch.cuda.stream(self._side):
            buf = torch.empty(shape, dtype=dtype, device=self.device)
            self.comm.recv(buf, peer)
        cur = torch.cuda.current_stream(self.device)
        cur.wait_stream(self._side)
        buf.record_stream(cur)
        return buf

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
        if self.first:
            xs = list(x.chunk(self.micro_batches))
            rows = [int(c.shape[0]) for c in xs]
        else:
            dt, trail, rows = self._recv_header(self.stage - 1)
        n_mb = len(rows)
        rows_total = target.shape[0] if self.last else None
        inputs, outputs, losses = [], [], []
        out_meta = None
        err = None  # a violation after the header went out: finish the step's protocol, then raise
        row = 0
        for i in range(n_mb):  # fill: all forwards
            if self.first:
                inp = xs[i].to(self.device, non_blocking=True)
            else:
                inp = self._recv((rows[i], *trail), dt, self.stage - 1)
                inp.requires_grad_(True)
            out = self.module(inp) if err is None else None
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
                continue
            if out is not None:
                why = None
                if out.dim() < 1 or out.shape[0] != rows[i]:
                    why = (f"PipelineStage {self.stage}: a stage must keep the row count "
                           f"({rows[i]} rows in, {tuple(out.shape)} out)")
                elif out_meta is not None and (out.dtype, tuple(out.shape[1:])) != out_meta:
                    why = (f"PipelineStage {self.stage}: micro-batch {i} output {(out.dtype, tuple(out.shape[1:]))} "
                           f"differs from micro-batch 0's {out_meta} (one step header per step)")
                if why is not None and out_meta is None:
                    raise RuntimeError(why)  # micro-batch 0: nothing sent yet
                err = why
            if out_meta is None:
                out_meta = (out.dtype, tuple(out.shape[1:]))
                self._send_header(_step_header(out, rows), self.stage + 1)
            if err is not None:  # the advertised payload, zeros: the next stage's step completes
                out = None
                self._send(torch.zeros((rows[i], *out_meta[1]), dtype=out_meta[0], device=self.device),
                           self.stage + 1)
            else:
                self._send(out, self.stage + 1)
            outputs.append(out)
        if self.last and row != rows_total:
            err = f"PipelineStage: received {row} rows for a target of {rows_total}"
        for i in reversed(range(len(outputs))):  # drain: backwards in reverse
            if self.last:
                if err is None:
                    outputs[i].backward()
            else:  # d(output): the shape and dtype of the activation this stage sent
                g = self._recv((rows[i], *out_meta[1]), out_meta[0], self.stage + 1)
                if outputs[i] is not None and err is None:
                    outputs[i].backward(g)
            if not self.first:
                gi = inputs[i].grad if err is None else None
                self._send(gi if gi is not None else torch.zeros_like(inputs[i]), self.stage - 1)
        self.synchronize()
        if err is not None:
            raise RuntimeError(err + " -- raised after completing the step's messages (no peer left waiting)")
        if self.last:
            return torch.stack([l.detach() for l in losses]).sum()
        return None

    @torch.no_grad()
    def forward(self, x: torch.Tensor | None = None) -> torch.Tensor | None:
        """Inference through the pipeline; returns the output on the last stage."""
        if self.first:
            inp = x.to(self.device)
        else:
            dt, trail, rows = self._recv_header(self.stage - 1)
            inp = self._recv((rows[0], *trail), dt, self.stage - 1)
        out = self.module(inp)
        if not self.last:
            self._send_header(_step_header(out, [int(out.shape[0])]), self.stage + 1)
            self._send(out, self.stage + 1)
            self.synchronize()
            return None
        return out
