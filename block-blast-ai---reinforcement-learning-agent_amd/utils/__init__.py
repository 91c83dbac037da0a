"""Training-driver utilities (logging, device selection, seeding)."""
from .device import get_device, set_seed  # noqa: F401
from .logger import Logger, MetricsTracker, TensorBoardLogger  # noqa: F401
