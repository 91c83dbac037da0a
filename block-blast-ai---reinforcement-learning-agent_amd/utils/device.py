"""Device selection and seeding (reference src/utils/device.py:9-90).

One process per GPU: under torch.distributed the device is ``cuda:LOCAL_RANK``.
The rollout path needs the HIP device — there is no CPU fallback, so
``get_device`` raises instead of silently returning the CPU.
"""
from __future__ import annotations

import os
import random
from typing import Optional

import numpy as np
import torch


def get_device(prefer_gpu: bool = True, gpu_id: Optional[int] = None, verbose: bool = True) -> torch.device:
    if not prefer_gpu:
        raise RuntimeError("the Block Blast rollout kernels need a HIP device (prefer_gpu=False is unsupported)")
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible: the MI355X build has no CPU rollout path")
    if gpu_id is None:
        gpu_id = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", gpu_id)
    torch.cuda.set_device(dev)
    if verbose:
        props = torch.cuda.get_device_properties(gpu_id)
        print(f"Using GPU {gpu_id}: {props.name} ({props.total_memory / 1e9:.1f} GB)")
    return dev


def set_seed(seed: int) -> None:
    """device.py:74-90: python, numpy global, torch (+ all devices)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
        torch.backends.cudnn.deterministic = True
        torch.backends.cudnn.benchmark = False
