"""Checkpoint / resume.

The reference never saves; this module adds the standard DDP pattern with the
reference's state_dict layout: rank 0 writes ``{"model", "optimizer", "epoch",
...}`` with ``torch.save`` (DDP-wrapped models keep the ``module.`` prefix),
every rank waits at a barrier, and resume restores the epoch so
``sampler.set_epoch`` continues the same permutation sequence. Files are
written atomically (tmp + rename) and loaded with ``weights_only=True``.
"""
from __future__ import annotations

import os

import torch


def _unwrap(sd: dict, prefix: str = "module.") -> dict:
    if sd and all(k.startswith(prefix) for k in sd):
        return {k[len(prefix):]: v for k, v in sd.items()}
    return sd


def save_checkpoint(path: str, model, optimizer=None, epoch: int = 0, rank: int = 0, extra: dict | None = None,
                    barrier=None) -> None:
    if rank == 0:
        state = {"model": model.state_dict(), "epoch": int(epoch)}
        if optimizer is not None:
            state["optimizer"] = optimizer.state_dict()
        if extra:
            state.update(extra)
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        tmp = path + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)
    if barrier is not None:
        barrier()


def load_checkpoint(path: str, model=None, optimizer=None, map_location="cpu", strict: bool = True) -> dict:
    state = torch.load(path, map_location=map_location, weights_only=True)
    if model is not None:
        sd = state["model"]
        target_keys = set(model.state_dict().keys())
        if not (set(sd) & target_keys):
            # accept a DDP checkpoint into a bare module and vice versa
            sd = _unwrap(sd) if any(k.startswith("module.") for k in sd) else {"module." + k: v for k, v in sd.items()}
        model.load_state_dict(sd, strict=strict)
    if optimizer is not None and "optimizer" in state:
        optimizer.load_state_dict(state["optimizer"])
    return state
