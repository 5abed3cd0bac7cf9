"""DDP toy job launched with ``mp.spawn`` -- one process per GPU.

Same entrypoint/CLI as the reference ``ddp_gpus.py``:
``python ddp_gpus.py --max_epochs 5 --batch_size 32``. ``world_size`` is the
number of visible GPUs (``--nprocs`` overrides, e.g. CPU/gloo runs). Rendezvous
on port 12345 like the reference (``PTDT_MASTER_PORT`` overrides, fixing quirk
Q6) at 127.0.0.1 instead of ``localhost`` (the hostname may not resolve in
containers; ``PTDT_MASTER_ADDR`` overrides).
"""
import torch

from pytorch_distributed_training_tutorials_amd.apps.ddp_toy import parser, run
from pytorch_distributed_training_tutorials_amd.parallel.env import ddp_setup, destroy_process_group
from pytorch_distributed_training_tutorials_amd.parallel.launcher import spawn


def main(rank: int, world_size: int, args):
    ddp_setup(rank, world_size)
    run(args, rank)
    destroy_process_group()


if __name__ == "__main__":
    p = parser()
    p.add_argument("--nprocs", type=int, default=None, help="ranks to spawn (default: visible GPUs)")
    args = p.parse_args()
    world_size = args.nprocs or max(torch.cuda.device_count(), 1)
    spawn(main, args=(world_size, args), nprocs=world_size)
