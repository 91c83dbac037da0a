"""Device-resident PPO training driver (reference scripts/train.py)."""
from .trainer import DEFAULT_CONFIG, DeviceRollout, create_directories, load_config, ppo_config_from, train  # noqa: F401
