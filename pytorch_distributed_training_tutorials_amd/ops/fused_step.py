"""Fused DDP train-step engine for Linear[-ReLU-Linear] models.

Reference hot loop (ddp_gpus.py:34-48): per step the
reference runs DataLoader collation, two H2D copies, ~10 tiny ATen kernels, the
DDP reducer's bucket copy + 84-byte NCCL all-reduce, and a foreach SGD -- a
purely latency-bound step. On MI355X this engine reduces one DDP step to

    fused_mlp_step kernel  (gather batch by sampler index -> fwd -> loss -> bwd
                            -> grads into the flat bucket, and the PREVIOUS
                            step's SGD update applied first)
    RCCL all-reduce(avg)   (the bucket, on the same stream)

and a chunk of steps is captured once into a hipGraph and replayed, so the
host issues one graph launch per chunk instead of ~15 launches per step. The
optimizer update of step s is applied at the start of step s+1's kernel (the
kernel reads the all-reduced bucket before overwriting it); the chunk's last
update is a single flat SGD launch, so after every replay the parameters are
exactly those of K full SGD steps.

The model keeps its ``nn.Linear`` parameters: they become views of the flat
parameter buffer, and their ``.grad`` views of the flat gradient bucket, so
``model.state_dict()`` / ``.grad`` inspection behave like the reference.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .._ext import native
from .flat import FlatParameters

LOSS_KINDS = {"ce_soft": 0, "ce_index": 1, "mse": 2}


def _linears(model: nn.Module):
    """Extract (layers, relu) for Linear / Sequential(Linear, ReLU, Linear) models."""
    mods = [m for m in model.modules() if not list(m.children())]
    lin = [m for m in mods if isinstance(m, nn.Linear)]
    relu = any(isinstance(m, nn.ReLU) for m in mods) or any(getattr(m, "relu", False) for m in lin[:1])
    if len(lin) == 1 and not relu:
        return lin, False
    if len(lin) == 2 and relu:
        return lin, True
    raise ValueError("FusedMLPStep supports Linear or Linear-ReLU-Linear models; use the autograd engine otherwise")


_VARIANTS = {"auto": 0, "workgroup": 1, "wave": 2, "wave_rows": 3, "wave_f": 4, "mfma": 5, "tp": 6, "tp_bf16": 7}
DTYPES = ("fp32", "bf16")


def _variant_id(variant: str | None) -> int:
    v = variant or os.environ.get("PTDT_PERSIST", "auto")
    if v not in _VARIANTS:
        raise ValueError(f"persistent engine variant must be one of {sorted(_VARIANTS)}, got {v!r}")
    return _VARIANTS[v]


class FusedMLPStep:
    def __init__(self, model: nn.Module, *, loss: str = "ce_soft", lr: float = 1e-2, momentum: float = 0.0,
                 dampening: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False, comm=None,
                 reduce: bool = True, defer_update: bool = True, ignore_index: int = -100, xgmi=None,
                 dtype: str = "fp32"):
        """``dtype="bf16"``: the persistent engine runs the step with torch.autocast(bfloat16)
        semantics on bf16 MFMA operands (fp32 master weights, momentum and SGD;
        csrc/kernels/mlp_tp_impl.h) -- Linear-ReLU-Linear models on the tensor-parallel engine only."""
        layers, relu = _linears(model)
        if dtype not in DTYPES:
            raise ValueError(f"dtype must be one of {DTYPES}, got {dtype!r}")
        self.dtype = dtype
        if dtype == "bf16" and not relu:
            raise ValueError("FusedMLPStep(dtype='bf16') runs Linear-ReLU-Linear models (the bf16 TP engine)")
        self.model = model
        self.layers = layers
        if loss not in LOSS_KINDS:
            raise ValueError(f"loss must be one of {list(LOSS_KINDS)}")
        self.loss_kind = LOSS_KINDS[loss]
        self.has_bias = all(l.bias is not None for l in layers)
        if not self.has_bias and any(l.bias is not None for l in layers):
            raise ValueError("FusedMLPStep: all layers need a bias or none")
        self.Din = layers[0].in_features
        self.H = layers[0].out_features if relu else 0
        self.Dout = layers[-1].out_features
        params = []
        for l in layers:
            params.append(l.weight)
            if self.has_bias:
                params.append(l.bias)
        dev = params[0].device
        if dev.type != "cuda":
            raise RuntimeError("FusedMLPStep is the GPU engine; use the autograd engine on CPU")
        self.device = dev
        self.flat = FlatParameters(params, with_grads=True)
        self.P = self.flat.flat()
        self.G = self.flat.flat_grad()
        self.lr, self.momentum, self.dampening = lr, momentum, dampening
        self.weight_decay, self.nesterov = weight_decay, nesterov
        self.mom = torch.zeros_like(self.P) if momentum != 0 else None
        self.opt_step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.comm = comm
        self.xgmi = xgmi if (reduce and xgmi is not None) else None  # in-kernel all-reduce + update
        self.reduce = reduce and comm is not None and self.xgmi is None
        self.defer = defer_update
        self.ignore_index = ignore_index
        self._pending = False
        self.loss_buf = torch.zeros(1, device=dev)
        self._C = native()
        lds = self._C.fused_mlp_lds_bytes(1, self.Din, self.H, self.Dout)
        if lds > 160 * 1024:
            raise ValueError("model too large for the single-workgroup fused step")

    # ------------------------------------------------------------------ steps
    def _kernel(self, X, Y, idx, B, loss_out, update_mode):
        ce_index = self.loss_kind == LOSS_KINDS["ce_index"]
        self._C.fused_mlp_step(X, None if ce_index else Y, Y if ce_index else None, idx, self.P, self.G,
                               self.mom, self.opt_step, loss_out, B, self.Din, self.H, self.Dout,
                               self.loss_kind, self.ignore_index, self.has_bias, 1.0, False, update_mode,
                               self.lr, self.momentum, self.dampening, self.weight_decay, self.nesterov,
                               self.xgmi.handle if self.xgmi is not None else None)

    def step(self, X: torch.Tensor, Y: torch.Tensor, idx: torch.Tensor | None, B: int,
             loss_out: torch.Tensor | None = None):
        """One DDP step on rows ``idx[:B]`` of the resident dataset ``(X, Y)``."""
        if self.dtype != "fp32":
            raise NotImplementedError("the per-step fused kernel is fp32; dtype='bf16' runs the persistent engine")
        lo = self.loss_buf if loss_out is None else loss_out
        if self.xgmi is not None:
            # ONE launch: fwd + loss + bwd + xGMI all-reduce + SGD update
            self._kernel(X, Y, idx, B, lo, 2)
            return
        self._kernel(X, Y, idx, B, lo, 1 if (self.defer and self._pending) else 0)
        if self.reduce:
            self.comm.all_reduce(self.G, "avg")
        if self.defer:
            self._pending = True
        else:
            self._apply()

    def _apply(self):
        self._C.sgd_flat_(self.P, self.G, self.mom, self.opt_step, self.lr, self.momentum, self.dampening,
                          self.weight_decay, self.nesterov, 1.0)

    def flush(self):
        """Apply the pending (deferred) optimizer update."""
        if self._pending:
            self._apply()
            self._pending = False

    def run(self, X, Y, idx: torch.Tensor, batches, losses: torch.Tensor | None = None):
        """Steps over ``batches`` = [(start, size)] of the index tensor, then flush."""
        for i, (start, size) in enumerate(batches):
            lo = losses[i:i + 1] if losses is not None else None
            self.step(X, Y, idx[start:start + size], size, lo)
        self.flush()

    # ------------------------------------------------------------ persistent engine
    def run_persistent(self, X, Y, n_steps: int, batch_size: int, sampler, cursor: torch.Tensor,
                       losses: torch.Tensor, max_steps_per_launch: int = 8192, stamps: torch.Tensor | None = None,
                       variant: str | None = None, idx: torch.Tensor | None = None, cursor_j: int = 0):
        """Run ``n_steps`` DDP steps in persistent launches: each step = gather ->
        fwd/loss/bwd -> all-reduce (in-kernel xGMI one-shot; identity at world 1)
        -> SGD. Two engines (``variant``, default ``$PTDT_PERSIST`` or "auto"):
        "wave" (csrc/kernels/linear_wave.hip: Linear(Din, Dout) models with
        B <= 64, one wave, weights/momentum/batch in registers) and "workgroup"
        (csrc/kernels/fused_mlp.hip: any Linear[-ReLU-Linear], state in LDS);
        "auto" picks the wave engine when it supports the configuration. ``sampler`` is a DeviceDistributedSampler
        (sharding/permutation parameters); ``cursor`` an int32[2] device tensor
        ``[epoch, step_in_epoch]`` advanced by the kernel; ``losses[i]`` receives
        step i's mean loss (``losses`` must hold ``min(n_steps, max_steps_per_launch)``).
        ``idx`` (int32, the epoch's index list, e.g. torch's DistributedSampler
        order from DeviceDataLoader.device_indices) replaces the in-kernel
        permutation; the steps must then stay inside that epoch, starting at
        step ``cursor_j``."""
        if self.xgmi is None and self.comm is not None and self.comm.world > 1:
            raise RuntimeError("the persistent engine needs the xGMI all-reduce for world > 1")
        ce_index = self.loss_kind == LOSS_KINDS["ce_index"]
        vid = self._vid(variant)
        X, padded = self._wave_input(X, batch_size, sampler, vid)
        done = 0
        while done < n_steps:
            n = min(max_steps_per_launch, n_steps - done)
            self._C.fused_mlp_persistent(
                X, None if ce_index else Y, Y if ce_index else None, self.P, self.G, self.mom, self.opt_step,
                batch_size, self.Din, self.H, self.Dout, self.loss_kind, self.ignore_index, self.has_bias,
                self.lr, self.momentum, self.dampening, self.weight_decay, self.nesterov,
                self.xgmi.handle if self.xgmi is not None else None, n, sampler.num_replicas, sampler.rank,
                sampler.num_samples, sampler.shuffle, sampler.seed, cursor, losses, stamps, vid, padded,
                idx, cursor_j + done if idx is not None else -1)
            done += n
        self._pending = False

    def persistent_plan(self, X, Y, batch_size: int, sampler, cursor: torch.Tensor, losses: torch.Tensor,
                        variant: str | None = None, idx: torch.Tensor | None = None,
                        stamps: torch.Tensor | None = None, idx_e0: int = 0):
        """A :meth:`run_persistent` launch resolved once (native ``PersistentPlan``):
        arguments validated, engine/kernel chosen, tensors held. ``plan.launch(n)``
        runs ``n <= losses.numel()`` steps from the device cursor with nothing but a
        ``hipLaunchKernel`` on the host. ``idx``: explicit index lists instead of
        the in-kernel permutation -- ``[num_samples]`` (one epoch; ``launch(n, j)``
        with ``j`` the step in it) or ``[E, num_samples]`` for epochs
        ``idx_e0 .. idx_e0+E-1`` (``launch(n, pos)`` with ``pos = epoch * S + step``,
        the launch staying inside those epochs)."""
        if self.xgmi is None and self.comm is not None and self.comm.world > 1:
            raise RuntimeError("the persistent engine needs the xGMI all-reduce for world > 1")
        ce_index = self.loss_kind == LOSS_KINDS["ce_index"]
        vid = self._vid(variant)
        X, padded = self._wave_input(X, batch_size, sampler, vid)
        self._pending = False
        # launch-to-launch cache of the epoch index lists (tags -1: empty): a launch
        # starting inside an already computed epoch copies its list
        stride = (sampler.num_samples + 3) // 4 * 4
        lcache = None
        if idx is None:
            lcache = torch.zeros(2 * stride + 2, dtype=torch.int32, device=self.device)
            lcache[-2:] = -1
        return self._C.PersistentPlan(
            X, None if ce_index else Y, Y if ce_index else None, self.P, self.G, self.mom, self.opt_step,
            batch_size, self.Din, self.H, self.Dout, self.loss_kind, self.ignore_index, self.has_bias,
            self.lr, self.momentum, self.dampening, self.weight_decay, self.nesterov,
            self.xgmi.handle if self.xgmi is not None else None, sampler.num_replicas, sampler.rank,
            sampler.num_samples, sampler.shuffle, sampler.seed, cursor, losses, stamps, vid, padded, idx, lcache,
            idx_e0)

    def _vid(self, variant: str | None) -> int:
        """Engine variant id; dtype="bf16" means the bf16 TP engine (and nothing else)."""
        if self.dtype == "bf16":
            if (variant or "tp_bf16") not in ("tp_bf16", "auto"):
                raise ValueError(f"dtype='bf16' runs the 'tp_bf16' persistent engine, not {variant!r}")
            return _VARIANTS["tp_bf16"]
        vid = _variant_id(variant)
        if vid == _VARIANTS["tp_bf16"]:
            raise ValueError("the 'tp_bf16' engine needs FusedMLPStep(dtype='bf16')")
        return vid

    def _wave_input(self, X, batch_size, sampler, vid):
        """The wave engine reads whole lane chunks (L lanes x K features per row):
        when L*K > Din, hand it a zero-padded copy of X (cached per tensor version)."""
        eng = self._C.persistent_engine(batch_size, self.Din, self.H, self.Dout, self.loss_kind,
                                        sampler.num_samples, sampler.num_replicas, vid, self.has_bias)
        if not eng.startswith("wave"):
            return X, False
        lanes, kp = int(eng.split("L")[1].split("R")[0]), int(eng.split("K")[1])
        width = (lanes or 4) * kp  # L0: layout F, 4 feature groups
        if width <= self.Din:
            return X, False
        key = (X.data_ptr(), X._version, tuple(X.shape), width)
        cached = getattr(self, "_xpad", None)
        if cached is None or cached[0] != key:
            xp = torch.zeros(X.shape[0], width, device=X.device, dtype=X.dtype)
            xp[:, :self.Din].copy_(X)
            cached = (key, xp[:, :self.Din])
            self._xpad = cached
        return cached[1], True

    def persistent_engine(self, batch_size: int, sampler, variant: str | None = None) -> str:
        """Which persistent engine :meth:`run_persistent` runs: "workgroup" or
        "wave:L<l>R<r>K<k>" (lanes per row, rows per lane group, features per lane)."""
        return self._C.persistent_engine(batch_size, self.Din, self.H, self.Dout, self.loss_kind,
                                         sampler.num_samples, sampler.num_replicas, self._vid(variant),
                                         self.has_bias)

    # ------------------------------------------------------------ optimizer state
    def export_optimizer_state(self, optimizer) -> None:
        """Write the engine's SGD state into ``optimizer`` in torch.optim.SGD layout
        (``state[p]['momentum_buffer']``, absent before the first step), so
        ``optimizer.state_dict()`` snapshots interchange with the autograd engine."""
        self.flush()
        first = int(self.opt_step.item()) == 0
        for g in optimizer.param_groups:
            for p in g["params"]:
                st = optimizer.state[p]
                st.pop("momentum_buffer", None)
                if self.mom is not None and not first:
                    _, off, k = self.flat.offsets[id(p)]
                    st["momentum_buffer"] = self.mom[off:off + k].view_as(p).clone()

    def import_optimizer_state(self, optimizer) -> None:
        """Load ``optimizer``'s torch.optim.SGD state (e.g. after
        ``optimizer.load_state_dict``) into the engine: momentum buffers into the
        flat momentum, the first-step flag from their presence."""
        self.flush()
        have = False
        for g in optimizer.param_groups:
            for p in g["params"]:
                buf = optimizer.state.get(p, {}).get("momentum_buffer")
                if buf is not None and self.mom is not None:
                    _, off, k = self.flat.offsets[id(p)]
                    self.mom[off:off + k].copy_(buf.reshape(-1))
                    have = True
        self.opt_step.fill_(1 if have else 0)

    def state_tensors(self) -> dict:
        """Device copies of everything a step reads and writes (params, momentum,
        step flag): a restore point for failure recovery."""
        return {k: v.clone() for k, v in (("P", self.P), ("mom", self.mom), ("opt_step", self.opt_step))
                if v is not None}

    def restore(self, st: dict) -> None:
        for k, v in st.items():
            getattr(self, k).copy_(v)
        self._pending = False

    # ------------------------------------------------------------ hipGraphs
    def state(self):
        return [t for t in (self.P, self.G, self.mom, self.opt_step) if t is not None]

    def graph(self, fn, warmup_fn=None, extra_state=()):
        """Capture ``fn()`` (which issues steps/flushes, e.g. :meth:`run`) into a
        hipGraph. ``warmup_fn`` (default ``fn``) runs once eagerly first (RCCL and
        allocator warm-up); all engine state plus ``extra_state`` tensors are
        restored afterwards, so capturing never changes the training trajectory.
        Returns a :class:`WatchedGraph` -- call ``.replay()``."""
        tensors = self.state() + [t for t in extra_state if t is not None]
        saved = [t.clone() for t in tensors]
        pending = self._pending
        stream = torch.cuda.Stream(self.device)
        stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(stream):
            (warmup_fn or fn)()
        torch.cuda.current_stream(self.device).wait_stream(stream)
        torch.cuda.synchronize(self.device)
        for t, v in zip(tensors, saved):
            t.copy_(v)
        self._pending = pending
        g = torch.cuda.CUDAGraph()
        rc = getattr(self.comm, "handle", None)
        before = rc.captured if rc is not None else 0
        with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
            fn()
        self._pending = pending
        torch.cuda.synchronize(self.device)
        return WatchedGraph(g, rc, (rc.captured - before) if rc is not None else 0)

    def capture(self, X, Y, idx_buf: torch.Tensor, batches, losses: torch.Tensor | None = None):
        """Graph of :meth:`run` over ``batches``; refresh ``idx_buf`` before each replay."""
        return self.graph(lambda: self.run(X, Y, idx_buf, batches, losses), extra_state=(losses,))


class WatchedGraph:
    """A captured hipGraph whose RCCL collectives the communicator's watchdog
    follows: each captured collective is followed in the graph by a device
    completion mark (csrc/comm/rccl_comm.cpp), and every :meth:`replay` declares
    the ``n_collectives`` marks it will produce, so a replay that stalls aborts
    the communicator after ``PTDT_COMM_TIMEOUT`` instead of hanging."""

    def __init__(self, graph, rccl, n_collectives: int):
        self.graph, self.rccl, self.n_collectives = graph, rccl, n_collectives

    def replay(self):
        self.graph.replay()
        if self.n_collectives and self.rccl is not None:
            self.rccl.expect_captured(self.n_collectives)

    def reset(self):
        self.graph.reset()

