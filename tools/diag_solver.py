"""Diagnostics (not product): per-env hand-search counters of bb_step.

Runs the random-policy rollout with BB_DEBUG_MODE=2 and reports the cycle
distribution of the wave-cooperative hand search (escalate_kernel), its
attempts / passes / slow passes, and the worst boards.
"""
import json
import os
import sys

os.environ["BB_DEBUG_MODE"] = str(int(os.environ.get("BB_DEBUG_MODE", "0")) | 2)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"))
sys.path.insert(0, REPO)

import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from runtime.device_env import DeviceEnvBatch  # noqa: E402


def main():
    n = int(os.environ.get("N", "65536"))
    steps = int(os.environ.get("STEPS", "60"))
    dev = torch.device("cuda", 0)
    env = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device=dev)
    env.reset()
    mb = torch.zeros((n, 3), dtype=torch.int64, device=dev)
    env.obs(mask_bits=mb)
    act = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
    env.random_actions(mb, act[0], step=0)
    buf = np.zeros((n, 4), dtype=np.uint64)
    rows = []
    per_step = []
    for t in range(steps):
        env.step(act[t & 1], next_action=act[(t + 1) & 1], policy_step=t + 1)
        env.lib.bb_debug_counters(env.handle, buf.ctypes.data_as(C.c_void_p))
        idx = np.nonzero(buf[:, 2] > 0)[0]
        if idx.size == 0:
            continue
        f = buf[idx, 1]
        cyc = buf[idx, 2].astype(np.int64)
        att = (f & np.uint64(0xFFFF)).astype(np.int64)
        passes = ((f >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.int64)
        slow = ((f >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.int64)
        slots = (f >> np.uint64(48)).astype(np.int64)
        w0 = buf[idx, 0]; w3 = buf[idx, 3]
        quick_c = (w0 & np.uint64(0xFFFFFFFF)).astype(np.int64); disj_c = (w0 >> np.uint64(32)).astype(np.int64)
        line_c = (w3 & np.uint64(0xFFFFFFFF)).astype(np.int64)
        line_t = (w3 >> np.uint64(32)).astype(np.int64)
        per_step.append((t, int(idx.size), int(cyc.max())))
        for k in range(idx.size):
            rows.append((int(cyc[k]), int(att[k]), int(passes[k]), int(slow[k]), int(slots[k]), int(quick_c[k]), t,
                         int(idx[k]), int(disj_c[k]), int(line_c[k]), int(line_t[k])))
    a = np.array([r[:5] for r in rows], dtype=np.int64)
    q = lambda v, p: float(np.percentile(v, p))  # noqa: E731
    out = {
        "n": n, "steps": steps, "searches": int(a.shape[0]),
        "cycles": {p: q(a[:, 0], p) for p in (50, 90, 99, 99.9, 100)},
        "attempts": {p: q(a[:, 1], p) for p in (50, 90, 99, 100)},
        "passes": {p: q(a[:, 2], p) for p in (50, 90, 99, 100)},
        "slow_passes": {p: q(a[:, 3], p) for p in (50, 90, 99, 100)},
        "frac_any_slow": float((a[:, 3] > 0).mean()),
        "cycles_by_slow_passes": {int(s): float(a[a[:, 3] == s, 0].mean()) for s in range(0, 6) if (a[:, 3] == s).any()},
        "per_step(t,n,max_cycles)": per_step[:12],
        "worst": [dict(zip(("cycles", "attempts", "passes", "slow", "max_slots", "quick_cyc", "step", "env",
                            "disjoint_cyc", "line_cyc", "line_tasks"), r))
                  for r in sorted(rows, key=lambda r: -r[0])[:15]],
        "totals_cycles": {"all": int(sum(r[0] for r in rows)), "quick": int(sum(r[5] for r in rows)),
                          "disjoint": int(sum(r[8] for r in rows)), "line": int(sum(r[9] for r in rows))},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
