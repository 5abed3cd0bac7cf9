"""``python -m pytorch_distributed_training_tutorials_amd.launch --nproc-per-node N script.py ...``
(torchrun-compatible single-node launcher; see parallel/launcher.py)."""
import sys

from .parallel.launcher import main

if __name__ == "__main__":
    sys.exit(main())
