"""DDP toy job for ``torchrun`` (or ``python -m pytorch_distributed_training_tutorials_amd.launch``).

Same entrypoint/CLI as the reference ``ddp_gpus_torchrun.py``:
``torchrun --nproc-per-node 4 ddp_gpus_torchrun.py --max_epochs 5 --batch_size 32``;
rank / local rank / world size come from the launcher's environment.
"""
import os

from pytorch_distributed_training_tutorials_amd.apps.ddp_toy import parser, run
from pytorch_distributed_training_tutorials_amd.parallel.env import ddp_setup, destroy_process_group


def main(args):
    ddp_setup()
    run(args, int(os.environ.get("LOCAL_RANK", 0)))
    destroy_process_group()


if __name__ == "__main__":
    main(parser().parse_args())
