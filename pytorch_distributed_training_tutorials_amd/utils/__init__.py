"""Trainer, checkpointing, metrics, tracing and fault injection."""
from .checkpoint import load_checkpoint, save_checkpoint  # noqa: F401
from .metrics import JsonlSink, scaling_efficiency  # noqa: F401
from .trainer import Trainer  # noqa: F401
