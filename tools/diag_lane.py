#!/usr/bin/env python3
"""Diagnostics (not product): how many hand draws the in-lane budgeted search
(BB_LANE_BUDGET) settles inside step_kernel vs parks for escalate_kernel, and
their cycle counts.  Prints JSON."""
import ctypes as C
import json
import os
import sys

os.environ["BB_DEBUG_MODE"] = str(int(os.environ.get("BB_DEBUG_MODE", "0")) | 2)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from runtime.device_env import DeviceEnvBatch  # noqa: E402


def main():
    n, warm, steps = int(os.environ.get("N", "65536")), int(os.environ.get("WARM", "40")), int(os.environ.get("STEPS", "20"))
    dev = torch.device("cuda", 0)
    env = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device=dev)
    env.reset()
    mb = torch.zeros((n, 3), dtype=torch.int64, device=dev)
    env.obs(mask_bits=mb)
    act = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
    env.random_actions(mb, act[0], step=0)
    buf = np.zeros((n, 4), dtype=np.uint64)
    lane_ok, lane_park, esc = [], [], []
    wave_tot = []
    draws = parked = 0
    for t in range(warm + steps):
        env.step(act[t & 1], next_action=act[(t + 1) & 1], policy_step=t + 1)
        env.lib.bb_debug_counters(env.handle, buf.ctypes.data_as(C.c_void_p))
        if t < warm:
            continue
        lane = buf[:, 0] > 0
        pk = buf[:, 2] > 0
        draws += int((lane | pk).sum())
        parked += int(pk.sum())
        lane_ok.extend(buf[lane & ~pk, 0].astype(np.int64).tolist())
        lane_park.extend(buf[lane & pk, 0].astype(np.int64).tolist())
        esc.extend(buf[pk, 2].astype(np.int64).tolist())
        e2 = np.where(pk, buf[:, 2].astype(np.int64), 0)
        wt = e2.reshape(-1, 8).sum(1)
        wave_tot.append(int(wt.max()))
    pc = lambda v: {p: float(np.percentile(v, p)) for p in (50, 90, 99, 100)} if len(v) else None  # noqa: E731
    print(json.dumps({"budget": os.environ.get("BB_LANE_BUDGET", "0"), "draws_per_step": draws / steps,
                      "parked_per_step": parked / steps, "lane_settled_cycles": pc(lane_ok),
                      "lane_parked_cycles": pc(lane_park), "escalate_cycles": pc(esc),
                      "escalate_wave_max_per_step": pc(wave_tot)}))


if __name__ == "__main__":
    main()
