#!/usr/bin/env python3
"""Diagnostics (not product): per-launch time of the bench kernel from a fresh reset, twice in one process.

The bench's 20-after-5 line reads ~3.5% under its steady state.  Two passes of K launches, each starting
from the same reset (env i seeded 42 + i), back to back: if the second pass's first launches are as slow as
the first pass's, the cost is the young-episode workload; if only the first pass's are, it is the GPU's
clock ramp.  Prints one JSON object: per-launch ms of both passes.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import torch  # noqa: E402

from runtime.device_env import DeviceEnvBatch  # noqa: E402

POLICY_SEED = 0xB10C


def main():
    n, T, K = 65536, 128, int(os.environ.get("K", "60"))
    dev = torch.device("cuda", 0)
    out = {}
    for p in range(2):
        e = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device=dev)
        e.reset()
        mb = torch.zeros((n, 3), dtype=torch.int64, device=dev)
        e.obs(mask_bits=mb)
        a = [torch.zeros(n, dtype=torch.int32, device=dev), torch.zeros(n, dtype=torch.int32, device=dev)]
        e.random_actions(mb, a[0], seed=POLICY_SEED, step=0)
        outs = (torch.zeros((T, n), dtype=torch.float32, device=dev), torch.zeros((T, n), dtype=torch.uint8, device=dev),
                torch.zeros((T, n), dtype=torch.uint8, device=dev), torch.zeros((T, n), dtype=torch.int32, device=dev),
                torch.zeros((T, n, 3), dtype=torch.int64, device=dev))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
        torch.cuda.synchronize()
        ev[0].record()
        for k in range(K):
            e.rollout(T, a[0], outs[0], outs[1], lines=outs[2], actions_out=outs[3], mask_out=outs[4],
                      next_action=a[1], policy_seed=POLICY_SEED, policy_step0=k * T)
            a.reverse()
            ev[k + 1].record()
        torch.cuda.synchronize()
        out[f"pass{p}"] = [round(ev[k].elapsed_time(ev[k + 1]), 4) for k in range(K)]
        e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
