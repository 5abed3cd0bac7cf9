"""Models of the reference tutorials (toy models, ResNet-50, model-parallel splits, Llama placement)."""
from .toy import SampleModel, ToyMLP, ToyModel, ddp_toy_model, model_size  # noqa: F401
