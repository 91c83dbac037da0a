#!/usr/bin/env python3
"""Diagnostics (not product): per-step bb_step duration (HIP events) and the
number of hand searches per step, to separate the search tail from the
fixed per-step cost.  Prints JSON."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from runtime.device_env import DeviceEnvBatch  # noqa: E402


def main():
    n = int(os.environ.get("N", "65536"))
    warm = int(os.environ.get("WARM", "20"))
    steps = int(os.environ.get("STEPS", "60"))
    dev = torch.device("cuda", 0)
    env = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device=dev)
    env.reset()
    mb = torch.zeros((n, 3), dtype=torch.int64, device=dev)
    env.obs(mask_bits=mb)
    act = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
    env.random_actions(mb, act[0], step=0)
    hand = torch.zeros(n, dtype=torch.int32, device=dev)
    ms, draws = [], []
    for t in range(warm + steps):
        env.snapshot(hand=hand)
        used = ((hand >> 18) & 7)
        # envs with two pieces used draw a new hand this step (random policy: always legal)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        env.step(act[t & 1], next_action=act[(t + 1) & 1], policy_step=t + 1)
        b.record()
        torch.cuda.synchronize()
        if t >= warm:
            ms.append(a.elapsed_time(b) * 1e3)
            u = used.cpu().numpy()
            draws.append(int(np.isin(u, [3, 5, 6]).sum()))
    ms = np.array(ms)
    out = {"n": n, "warm": warm, "steps": steps, "us_mean": float(ms.mean()), "us_median": float(np.median(ms)),
           "us_max": float(ms.max()), "us_min": float(ms.min()),
           "per_step": [(round(float(x), 1), d) for x, d in zip(ms, draws)]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
