"""Process-group setup and the launcher environment contract.

Reference:
* spawn flavour ``ddp_setup(rank, world_size)`` ddp_gpus.py:12-17 -- hard-codes
  ``MASTER_ADDR=localhost``, ``MASTER_PORT=12345``, ``init_process_group("nccl",
  rank, world_size)``, ``torch.cuda.set_device(rank)``;
* torchrun flavour ``ddp_setup()`` ddp_gpus_torchrun.py:12-14 -- everything from
  the env (``RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT``);
* ``destroy_process_group()`` ddp_gpus.py:93.

Here ``init_process_group`` brings up torch's c10d group (env:// TCPStore
rendezvous) with ``cpu:gloo,cuda:nccl`` on GPU machines -- gloo is the cheap
host control plane (barriers, object broadcast, fingerprint checks) and
``nccl`` is RCCL for any user code calling ``torch.distributed`` on GPU
tensors -- and the framework's own native RCCL communicator for the hot path
is created lazily on top of the same store (``parallel.comm``). On CPU-only
hosts the backend is gloo (plumbing tests).
"""
from __future__ import annotations

import datetime as _dt
import os
import socket

import torch
import torch.distributed as dist


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def rank() -> int:
    return dist.get_rank() if is_initialized() else _env_int("RANK", 0)


def world_size() -> int:
    return dist.get_world_size() if is_initialized() else _env_int("WORLD_SIZE", 1)


def local_rank() -> int:
    return _env_int("LOCAL_RANK", rank())


def local_world_size() -> int:
    return _env_int("LOCAL_WORLD_SIZE", world_size())


def device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", local_rank() % max(torch.cuda.device_count(), 1))
    return torch.device("cpu")


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def default_backend() -> str:
    return "cpu:gloo,cuda:nccl" if torch.cuda.is_available() else "gloo"


def init_process_group(backend: str | None = None, rank: int | None = None, world_size: int | None = None,
                       timeout_s: float = 1800.0, device_id: int | None = None) -> None:
    """``torch.distributed.init_process_group`` with MI355X defaults.

    ``backend="nccl"`` (the reference's string) maps to ``cpu:gloo,cuda:nccl``
    on GPU hosts (RCCL for device tensors + a host control plane) and to
    ``gloo`` on CPU-only hosts. A missing rendezvous env (single-process run
    without a launcher) becomes a 1-rank group on 127.0.0.1.
    """
    if is_initialized():
        return
    if backend in (None, "nccl", "rccl"):
        backend = default_backend()
    if world_size is None:
        world_size = _env_int("WORLD_SIZE", 1)
    if rank is None:
        rank = _env_int("RANK", 0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        if world_size != 1:
            raise RuntimeError("MASTER_PORT is not set for a multi-process group")
        os.environ["MASTER_PORT"] = str(free_port())
    if torch.cuda.is_available():
        dev = device_id if device_id is not None else _env_int("LOCAL_RANK", rank) % torch.cuda.device_count()
        torch.cuda.set_device(dev)
    dist.init_process_group(backend=backend, rank=rank, world_size=world_size,
                            timeout=_dt.timedelta(seconds=timeout_s))


def destroy_process_group() -> None:
    from . import comm

    comm.destroy_all()
    if is_initialized():
        dist.destroy_process_group()


def ddp_setup(rank: int | None = None, world_size: int | None = None, *, master_addr: str = "127.0.0.1",
              master_port: str | int = "12345", backend: str | None = "nccl") -> None:
    """Both reference flavours in one call.

    * ``ddp_setup(rank, world_size)`` -- spawn flavour (ddp_gpus.py:12-17): sets
      ``MASTER_ADDR``/``MASTER_PORT`` (defaults localhost:12345 like the reference;
      ``PTDT_MASTER_PORT`` overrides the port, fixing quirk Q6) and selects
      ``cuda:rank``.
    * ``ddp_setup()`` -- torchrun flavour (ddp_gpus_torchrun.py:12-14): all from env.
    """
    if rank is not None:
        os.environ["MASTER_ADDR"] = os.environ.get("PTDT_MASTER_ADDR", master_addr)
        os.environ["MASTER_PORT"] = str(os.environ.get("PTDT_MASTER_PORT", master_port))
        os.environ["RANK"] = str(rank)
        os.environ["WORLD_SIZE"] = str(world_size)
        os.environ.setdefault("LOCAL_RANK", str(rank))
        init_process_group(backend, rank=rank, world_size=world_size, device_id=rank if torch.cuda.is_available() else None)
    else:
        init_process_group(backend)


def barrier() -> None:
    if is_initialized():
        from . import comm

        comm.get_default().barrier()
