"""Process groups, the native communicator, and the parallelism wrappers."""
from . import bucketing, comm, env  # noqa: F401
from .comm import Communicator, get_default  # noqa: F401
from .ddp import DistributedDataParallel  # noqa: F401
from .env import barrier, ddp_setup, destroy_process_group, init_process_group  # noqa: F401
