#!/usr/bin/env python3
"""Diagnostics (not product): step_kernel phase timestamps (BB_DEBUG_MODE=4):
table staging, state loads + validity, move, hand draw / in-lane search,
finalize -- per lane cycles, and the per-wave maxima that set the time."""
import ctypes as C
import json
import os
import sys

os.environ["BB_DEBUG_MODE"] = "4"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from runtime.device_env import DeviceEnvBatch  # noqa: E402


def main():
    n, warm, steps = int(os.environ.get("N", "65536")), int(os.environ.get("WARM", "40")), int(os.environ.get("STEPS", "10"))
    dev = torch.device("cuda", 0)
    env = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device=dev)
    env.reset()
    mb = torch.zeros((n, 3), dtype=torch.int64, device=dev)
    env.obs(mask_bits=mb)
    act = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
    env.random_actions(mb, act[0], step=0)
    buf = np.zeros((n, 4), dtype=np.uint64)
    rows = []
    for t in range(warm + steps):
        env.step(act[t & 1], next_action=act[(t + 1) & 1], policy_step=t + 1)
        env.lib.bb_debug_counters(env.handle, buf.ctypes.data_as(C.c_void_p))
        if t < warm:
            continue
        w0, w1 = buf[:, 0], buf[:, 1]
        ph = np.stack([(w0 >> np.uint64(16 * k)) & np.uint64(0xFFFF) for k in range(4)] +
                      [(w1 >> np.uint64(16)) & np.uint64(0xFFFF)], 1).astype(np.int64)
        kind = (w1 & np.uint64(0xFF)).astype(np.int64)      # 1 parked, 2 finalized
        drew = ((w1 >> np.uint64(8)) & np.uint64(1)).astype(np.int64)
        rows.append((ph, kind, drew))
    ph = np.concatenate([r[0] for r in rows])
    kind = np.concatenate([r[1] for r in rows])
    drew = np.concatenate([r[2] for r in rows])
    names = ["stage", "load+valid", "move", "draw/search", "finalize"]
    pc = lambda v: {p: float(np.percentile(v, p)) for p in (50, 90, 99, 100)}  # noqa: E731
    out = {"n": n, "lanes": int(ph.shape[0]), "frac_parked": float((kind == 1).mean()),
           "frac_drew": float(((kind == 2) & (drew == 1)).mean() + (kind == 1).mean())}
    for k, nm in enumerate(names):
        out[nm] = pc(ph[:, k])
    # per-wave (64 consecutive lanes) max of the total
    tot = ph.sum(1)
    waves = tot[: (tot.size // 64) * 64].reshape(-1, 64).max(1)
    out["wave_total_max_cycles"] = pc(waves)
    sr = ph[:, 3][: (tot.size // 64) * 64].reshape(-1, 64).max(1)
    out["wave_search_max_cycles"] = pc(sr)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
