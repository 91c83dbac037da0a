#!/usr/bin/env python3
"""Diagnostics (not product): finalize sub-phases in step_kernel
(BB_DEBUG_MODE=8): masks, reward, info+outputs, auto-reset/state stores,
mask/policy outputs -- per-lane cycles and per-wave maxima."""
import ctypes as C
import json
import os
import sys

os.environ["BB_DEBUG_MODE"] = "8"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from runtime.device_env import DeviceEnvBatch  # noqa: E402


def main():
    n, warm, steps = int(os.environ.get("N", "65536")), 40, 10
    dev = torch.device("cuda", 0)
    env = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device=dev)
    env.reset()
    mb = torch.zeros((n, 3), dtype=torch.int64, device=dev)
    env.obs(mask_bits=mb)
    act = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
    env.random_actions(mb, act[0], step=0)
    buf = np.zeros((n, 4), dtype=np.uint64)
    ph = []
    for t in range(warm + steps):
        env.step(act[t & 1], next_action=act[(t + 1) & 1], policy_step=t + 1)
        env.lib.bb_debug_counters(env.handle, buf.ctypes.data_as(C.c_void_p))
        if t >= warm:
            w2, w3 = buf[:, 2], buf[:, 3]
            ph.append(np.stack([(w2 >> np.uint64(16 * k)) & np.uint64(0xFFFF) for k in range(4)] +
                               [w3 & np.uint64(0xFFFFFFFF)], 1).astype(np.int64))
    ph = np.concatenate(ph)
    names = ["masks", "reward", "info+outputs", "reset/stores", "policy"]
    pc = lambda v: {p: float(np.percentile(v, p)) for p in (50, 90, 99, 100)}  # noqa: E731
    out = {nm: pc(ph[:, k]) for k, nm in enumerate(names)}
    w = ph[: (len(ph) // 64) * 64].reshape(-1, 64, 5).max(1)
    out["wave_max_sum"] = pc(w.sum(1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
