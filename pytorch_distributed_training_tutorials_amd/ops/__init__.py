"""Native (gfx950 HIP) operators with autograd and CPU reference fallbacks."""
from .flat import FlatParameters, contiguous_span  # noqa: F401
from .fused_step import FusedMLPStep  # noqa: F401
from .linear import Linear, gemm, linear  # noqa: F401
from .loss import CrossEntropyLoss, MSELoss, cross_entropy, mse_loss  # noqa: F401
from .optim import FusedAdam, FusedSGD  # noqa: F401
