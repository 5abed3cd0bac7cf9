"""Trainer with the reference's public surface.

Reference: ``Trainer(model, train_dataloader, optimizer, gpu_id)`` and
``.train(max_epoch)`` (ddp_gpus.py:19-53, ddp_gpus_torchrun.py:16-49; SURVEY R6,
R14): moves the model to the GPU, wraps it in DDP, and per epoch prints
``[GPU: {gpu_id} Epoch: {epoch}, Batch size: {batch_size} | Steps {steps}]``,
calls ``sampler.set_epoch(epoch)`` and runs zero_grad -> forward ->
cross_entropy -> backward -> step per batch.

Engines (same observable result, different execution):
  * ``persistent`` -- GPU, Linear[-ReLU-Linear] models + SGD, one rank or a
                    working in-kernel xGMI all-reduce: ONE kernel launch runs
                    every DDP step of every epoch up to the next snapshot
                    (ops/fused_step.py persistent_plan; the single-wave engine
                    for Linear models), fed the torch-identical
                    DistributedSampler orders of all those epochs, computed on
                    the GPU by one launch (data/torch_perm.py). The status lines
                    of the launched epochs are printed before it. After it the
                    xGMI error flag is read at the closing sync and agreed across
                    ranks; on a timed-out poll every rank restores the launch's
                    starting parameters and re-runs those epochs on the fused
                    engine with RCCL. The default whenever available.
  * ``fused``    -- GPU, Linear[-ReLU-Linear] models + SGD: one fused kernel +
                    one RCCL all-reduce per step, a whole epoch captured into a
                    hipGraph and replayed (ops/fused_step.py). The default on GPU
                    whenever the model/optimizer/loss allow it.
  * ``autograd`` -- any model: native DDP reducer (bucketed RCCL all-reduce
                    overlapped with backward) + native kernels for Linear / loss /
                    optimizer where applicable; CPU/gloo for plumbing tests.
Extras: rank-0 snapshots every ``save_every`` epochs with resume
(``snapshot_path``; every engine saves its optimizer state in torch.optim.SGD
layout, so snapshots interchange between engines), fault injection hooks,
JSONL metrics.
"""
from __future__ import annotations

import os
import time

import torch
import torch.nn as nn

from .._ext import native
from ..data.loader import DeviceDataLoader
from ..ops.fused_step import FusedMLPStep, _linears
from ..ops.loss import cross_entropy
from ..parallel import comm as comm_mod
from ..parallel import env
from ..parallel.ddp import DistributedDataParallel, _flatten_broadcast
from .checkpoint import load_checkpoint, save_checkpoint
from .faults import FaultInjector
from .metrics import JsonlSink
from .tracing import trace


class _ModuleView(nn.Module):
    """DDP-shaped container (``module.`` state_dict prefix) for the fused engine."""

    def __init__(self, module):
        super().__init__()
        self.module = module

    def forward(self, *a, **k):
        return self.module(*a, **k)


class _Shard:
    """Sampler parameters the persistent kernel needs when it is given the index list."""

    def __init__(self, world, rank, num_samples):
        self.num_replicas, self.rank, self.num_samples = world, rank, num_samples
        self.shuffle, self.seed = False, 0


def _sgd_hparams(opt):
    g = opt.param_groups[0]
    if len(opt.param_groups) != 1 or "momentum" not in g:
        return None
    if type(opt).__name__ not in ("SGD", "FusedSGD") or g.get("maximize", False):
        return None
    return dict(lr=g["lr"], momentum=g.get("momentum", 0.0), dampening=g.get("dampening", 0.0),
                weight_decay=g.get("weight_decay", 0.0), nesterov=g.get("nesterov", False))


class Trainer:
    def __init__(self, model: nn.Module, train_dataloader, optimizer: torch.optim.Optimizer, gpu_id: int | None = None,
                 *, loss_fn=None, engine: str = "auto", graph: bool = True, comm=None,
                 snapshot_path: str | None = None, save_every: int = 0, metrics_path: str | None = None,
                 log=print, ddp_kwargs: dict | None = None, verbose: bool = True):
        self.gpu_id = env.local_rank() if gpu_id is None else gpu_id
        self.device = torch.device("cuda", self.gpu_id) if torch.cuda.is_available() else torch.device("cpu")
        self.rank = env.rank()
        self.world_size = env.world_size()
        self.train_dataloader = train_dataloader
        self.optimizer = optimizer
        self.loss_fn = loss_fn or cross_entropy
        self.log = log if verbose else (lambda *a, **k: None)
        self.graph = graph
        self.snapshot_path = snapshot_path
        self.save_every = save_every
        self.epochs_run = 0
        self.global_step = 0
        self.faults = FaultInjector(self.rank)
        self.metrics = JsonlSink(metrics_path, self.rank)
        self.comm = comm if comm is not None else comm_mod.get_default(self.device if self.device.type == "cuda" else None)
        model = model.to(self.device)
        self.engine_name = self._select_engine(engine, model)
        self.xgmi = None
        self.fallbacks = []  # (epoch range, reason) of every xGMI -> RCCL fallback
        xg = None
        if self.engine_name == "persistent" and self.world_size > 1:
            from ..parallel.xgmi import maybe_create

            xg = maybe_create(self.comm, self.device)  # collective: every rank takes this branch
            self.xgmi = xg
            if xg is None:
                if engine == "persistent":
                    raise RuntimeError("persistent engine: the in-kernel xGMI all-reduce is unavailable")
                self.engine_name = "fused"
        if self.engine_name in ("fused", "persistent"):
            hp = _sgd_hparams(optimizer)
            loss_kind = self._fused_loss_kind()
            self.engine = FusedMLPStep(model, loss=loss_kind, comm=self.comm, xgmi=xg, **hp)
            if self.world_size > 1:  # DDP init semantics: rank 0's parameters everywhere (M4)
                self.comm.broadcast(self.engine.P, 0)
            self.model = _ModuleView(model)
            self._idx_buf = None
            self._graphs = {}
            self._loss_buf = None
            self._cursor = None
        else:
            self.engine = None
            self.model = DistributedDataParallel(model, device_ids=[self.gpu_id] if self.device.type == "cuda" else None,
                                                 comm=self.comm, **(ddp_kwargs or {}))
        if snapshot_path and os.path.exists(snapshot_path):
            self._load_snapshot(snapshot_path)

    # ------------------------------------------------------------ engine choice
    def _fusable(self, model) -> bool:
        if self.device.type != "cuda" or not isinstance(self.train_dataloader, DeviceDataLoader):
            return False
        dl = self.train_dataloader
        if dl.drop_last and dl._num_samples() % dl.batch_size:
            return False  # the engines run ceil(num_samples / B) steps with a short last batch
        if self.loss_fn is not cross_entropy and getattr(self.loss_fn, "__name__", "") not in ("cross_entropy", "mse_loss"):
            return False
        if _sgd_hparams(self.optimizer) is None:
            return False
        try:
            _linears(model)
        except ValueError:
            return False
        return True

    def _select_engine(self, engine: str, model) -> str:
        if engine == "auto":
            return "persistent" if self._fusable(model) else "autograd"
        if engine in ("fused", "persistent") and not self._fusable(model):
            raise ValueError(f"{engine} engine needs: GPU, DeviceDataLoader, SGD, Linear[-ReLU-Linear], CE/MSE loss")
        return engine

    def _fused_loss_kind(self) -> str:
        if getattr(self.loss_fn, "__name__", "") == "mse_loss":
            return "mse"
        y = self.train_dataloader.dataset.tensors[1]
        return "ce_soft" if y.is_floating_point() else "ce_index"

    # ------------------------------------------------------------ reference API
    def _run_batch(self, xs, ys):
        self.optimizer.zero_grad()
        with trace("fwd"):
            output = self.model(xs)
            loss = self.loss_fn(output, ys)
        with trace("bwd"):
            loss.backward()
        with trace("opt"):
            self.optimizer.step()
        return loss

    def _first_batch_size(self) -> int:
        dl = self.train_dataloader
        n = len(dl.sampler) if getattr(dl, "sampler", None) is not None else len(dl.dataset)
        return min(dl.batch_size, n)

    def _set_epoch(self, epoch: int):
        dl = self.train_dataloader
        if isinstance(dl, DeviceDataLoader):
            dl.set_epoch(epoch)
        elif getattr(dl, "sampler", None) is not None and hasattr(dl.sampler, "set_epoch"):
            dl.sampler.set_epoch(epoch)

    def _run_epoch(self, epoch: int):
        b_sz = self._first_batch_size()
        self.log(f"[GPU: {self.gpu_id} Epoch: {epoch}, Batch size: {b_sz} | Steps {len(self.train_dataloader)}]")
        self._set_epoch(epoch)
        t0 = time.perf_counter()
        if self.engine_name in ("fused", "persistent"):
            self._run_epoch_fused()
        else:
            for xs, ys in self.train_dataloader:
                xs = xs.to(self.device, non_blocking=True)
                ys = ys.to(self.device, non_blocking=True)
                self.faults.check(self.global_step)
                self._run_batch(xs, ys)
                self.global_step += 1
        if self.metrics.enabled:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self.metrics.write(event="epoch", epoch=epoch, seconds=time.perf_counter() - t0,
                               steps=len(self.train_dataloader), engine=self.engine_name)

    # ------------------------------------------------------------ fused engine
    def _run_epoch_fused(self):
        dl = self.train_dataloader
        ds = dl.dataset
        X, Y = ds.tensors[0], ds.tensors[1]
        n = dl._num_samples()
        if self._idx_buf is None:
            self._idx_buf = torch.zeros(n, dtype=torch.int32, device=self.device)
        dl.device_indices(out=self._idx_buf)
        batches = tuple(dl.batches())
        if self._loss_buf is None or self._loss_buf.numel() < len(batches):
            self._loss_buf = torch.zeros(len(batches), device=self.device)
        if os.environ.get("PTDT_FAULT_RANK") is not None:  # per step on every rank (same collectives)
            for i, (s, b) in enumerate(batches):
                self.faults.check(self.global_step + i)
                self.engine.step(X, Y, self._idx_buf[s:s + b], b, self._loss_buf[i:i + 1])
            self.engine.flush()
        elif self.graph:
            g = self._graphs.get(batches)
            if g is None:
                g = self.engine.capture(X, Y, self._idx_buf, list(batches), self._loss_buf)
                self._graphs[batches] = g
            g.replay()
        else:
            self.engine.run(X, Y, self._idx_buf, list(batches), self._loss_buf)
        self.global_step += len(batches)

    # ------------------------------------------------------------ persistent engine
    def _run_epochs_persistent(self, e0: int, e1: int):
        """Epochs [e0, e1) in ONE persistent launch (status lines first)."""
        dl = self.train_dataloader
        X, Y = dl.dataset.tensors[0], dl.dataset.tensors[1]
        n = dl._num_samples()
        S = len(dl)
        E = e1 - e0
        b_sz = self._first_batch_size()
        for epoch in range(e0, e1):
            self.log(f"[GPU: {self.gpu_id} Epoch: {epoch}, Batch size: {b_sz} | Steps {S}]")
        t0 = time.perf_counter()
        dl.set_epoch(e1 - 1)  # the loader/sampler end where the reference's would
        lists = dl.device_epoch_indices(range(e0, e1))  # torch-identical orders, one launch
        if self._loss_buf is None or self._loss_buf.numel() < E * S:
            self._loss_buf = torch.zeros(E * S, device=self.device)
        if self._cursor is None:
            self._cursor = torch.zeros(2, dtype=torch.int32, device=self.device)
        self._cursor.copy_(torch.tensor([e0, 0], dtype=torch.int32), non_blocking=True)
        restore = self.engine.state_tensors() if self.xgmi is not None else None
        shard = _Shard(self.world_size, self.rank, n)
        plan = self.engine.persistent_plan(X, Y, dl.batch_size, shard, self._cursor, self._loss_buf[:E * S],
                                           idx=lists, idx_e0=e0)
        plan.launch_at(E * S, e0 * S)  # start position from the arguments (the cursor copy is for the end state)
        self.global_step += E * S
        if self.xgmi is not None and self._xgmi_failed():
            self._fallback_to_rccl(e0, e1, restore)
        if self.metrics.enabled:
            torch.cuda.synchronize(self.device)
            self.metrics.write(event="epochs", first=e0, last=e1 - 1, seconds=time.perf_counter() - t0,
                               steps=E * S, engine=self.engine_name)

    def _max_epochs_per_launch(self) -> int:
        """Epochs one persistent launch may cover: its epoch lists ([E, num_samples] int32),
        the torch_perm workspace (E * 4n int32 when the permutation state does not fit
        in LDS) and the loss slots grow with E, so E is bounded by a device-memory budget
        (``PTDT_PERSIST_EPOCH_BYTES``, default 256 MiB) instead of by ``max_epoch``."""
        dl = self.train_dataloader
        n, ns, S = len(dl.dataset), dl._num_samples(), len(dl)
        per_epoch = 4 * ns + 4 * S
        if native().torch_perm_needs_ws(n):
            per_epoch += 16 * n
        budget = int(os.environ.get("PTDT_PERSIST_EPOCH_BYTES", 256 << 20))
        return max(1, budget // per_epoch)

    def _xgmi_failed(self) -> bool:
        """Did any rank's in-kernel all-reduce time out a poll? Read at the launch's
        closing sync (one flag read per launch, none per step) and agreed by a
        max-reduction, so every rank takes the same branch."""
        bad = torch.tensor([float(self.xgmi.handle.error() != 0)], device=self.device)
        self.comm.all_reduce(bad, "max")
        return bad.item() != 0

    def _fallback_to_rccl(self, e0: int, e1: int, restore: dict):
        """A peer never arrived in the in-kernel all-reduce: replicas may hold
        garbage. Every rank restores the launch's starting state, re-broadcasts
        rank 0's parameters, drops the xGMI path and re-runs the epochs on the
        fused engine with the RCCL all-reduce."""
        msg = (f"[ptdt] rank {self.rank}: xGMI all-reduce timed out in epochs {e0}-{e1 - 1}; restoring their "
               f"starting parameters and re-running them on the fused engine with RCCL")
        print(msg, flush=True)
        self.fallbacks.append(((e0, e1), "xgmi poll timeout"))
        self.engine.restore(restore)
        self.comm.broadcast(self.engine.P, 0)
        if self.engine.mom is not None:
            self.comm.broadcast(self.engine.mom, 0)
        self.xgmi.handle.reset_error()
        self.xgmi = None
        self.engine.xgmi = None
        self.engine.reduce = True
        self.engine_name = "fused"
        self._graphs = {}
        self.global_step -= (e1 - e0) * len(self.train_dataloader)
        for epoch in range(e0, e1):  # status lines were printed before the failed launch
            self._set_epoch(epoch)
            self._run_epoch_fused()

    def last_losses(self) -> torch.Tensor | None:
        return None if self._loss_buf is None else self._loss_buf

    # ------------------------------------------------------------ snapshots
    def _save_snapshot(self, epoch: int):
        if self.engine is not None:  # torch.optim.SGD layout: snapshots interchange between engines
            self.engine.export_optimizer_state(self.optimizer)
        save_checkpoint(self.snapshot_path, self.model, self.optimizer, epoch=epoch, rank=self.rank,
                        barrier=self.comm.barrier)

    def _load_snapshot(self, path: str):
        st = load_checkpoint(path, self.model, self.optimizer, map_location=self.device)
        if self.engine is not None:
            self.engine.import_optimizer_state(self.optimizer)
        self.epochs_run = int(st.get("epoch", -1)) + 1
        self.log(f"Resuming training from snapshot at Epoch {self.epochs_run}")

    def _save_due(self, epoch: int) -> bool:
        return bool(self.snapshot_path and self.save_every and (epoch + 1) % self.save_every == 0)

    def train(self, max_epoch: int):
        epoch = self.epochs_run
        # fault injection runs per step on EVERY rank (one rank alone on another engine would desync)
        per_step = os.environ.get("PTDT_FAULT_RANK") is not None
        while epoch < max_epoch:
            if self.engine_name == "persistent" and not per_step:
                end = min(max_epoch, epoch + self._max_epochs_per_launch())
                if self.snapshot_path and self.save_every:  # one launch per snapshot interval
                    end = min(end, (epoch // self.save_every + 1) * self.save_every)
                self._run_epochs_persistent(epoch, end)
                epoch = end
            else:
                self._run_epoch(epoch)
                epoch += 1
            if self._save_due(epoch - 1):
                self._save_snapshot(epoch - 1)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
