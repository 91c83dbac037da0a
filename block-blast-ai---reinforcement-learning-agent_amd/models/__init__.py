"""Policy/value network (PyTorch-ROCm)."""
from .network import BlockBlastNetwork, ResidualBlock, count_params  # noqa: F401
