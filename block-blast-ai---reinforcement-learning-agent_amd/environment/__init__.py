"""Gym surface (BlockBlastEnv, VectorizedBlockBlastEnv) over the HIP vec-env."""
from .block_blast_env import BlockBlastEnv, BlockBlastEnvFlat  # noqa: F401
from .extra_wrappers import FrameStackWrapper, NormalizedRewardWrapper, RunningMeanStd, make_env  # noqa: F401
from .wrappers import VectorizedBlockBlastEnv  # noqa: F401
