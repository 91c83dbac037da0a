"""Masked-PPO agent (rollout kernels on HIP, update in PyTorch-ROCm + RCCL)."""
from .base import BaseAgent  # noqa: F401
from .ppo import PackedRolloutBuffer, PPOAgent, PPOConfig, RolloutBuffer, broadcast_parameters  # noqa: F401
