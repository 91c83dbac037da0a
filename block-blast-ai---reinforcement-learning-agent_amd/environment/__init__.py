"""Gym surface (BlockBlastEnv, VectorizedBlockBlastEnv) over the HIP vec-env."""
from .block_blast_env import BlockBlastEnv, BlockBlastEnvFlat  # noqa: F401
from .wrappers import VectorizedBlockBlastEnv  # noqa: F401
