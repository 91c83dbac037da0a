"""Diagnostics (not product): where the rollout tail comes from.

Needs the -DBB_ROLL_DIAG=3 build (BBVEC_LIB=...) and BB_DEBUG_MODE=16.  For
two consecutive rollout launches, per wave: busy cycles (sum of phases), span
(s_memrealtime, 10 ns ticks), start offset, and placement (XCC, SE, CU, SIMD
from HW_ID).  Reports whether slow waves are slow again in the next launch
(group- or placement-bound) and how busy each SIMD's wave pair is.
"""
import ctypes as C
import json
import os
import sys

os.environ["BB_DEBUG_MODE"] = "16"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from runtime.device_env import DeviceEnvBatch  # noqa: E402


def main():
    n, T, W = 65536, int(os.environ.get("T", "128")), 18
    dev = torch.device("cuda", 0)
    env = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device=dev)
    env.reset()
    mb = torch.zeros((n, 3), dtype=torch.int64, device=dev)
    env.obs(mask_bits=mb)
    act = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
    env.random_actions(mb, act[0], step=0)
    rew = torch.zeros((T, n), dtype=torch.float32, device=dev)
    term = torch.zeros((T, n), dtype=torch.uint8, device=dev)
    buf = np.zeros((n, 4), dtype=np.uint64)
    runs = []
    for call in range(4):
        env.rollout(T, act[0], rew, term, next_action=act[1], policy_step0=call * T)
        act.reverse()
        torch.cuda.synchronize()
        env.lib.bb_debug_counters(env.handle, buf.ctypes.data_as(C.c_void_p))
        w = buf.reshape(-1)[: (n // 32) * W].reshape(-1, W).astype(np.int64)
        runs.append(w)
    out = {}
    a, b = runs[2], runs[3]
    busy_a = a[:, 0] + a[:, 1] + a[:, 2]
    busy_b = b[:, 0] + b[:, 1] + b[:, 2]
    span_a = a[:, 17] - a[:, 16]
    start_a = a[:, 16] - a[:, 16].min()
    hw = a[:, 15] & 0xFFFFFFFF
    xcc = (a[:, 15] >> 32) & 0xF
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
    out["busy_corr_next_launch"] = float(np.corrcoef(busy_a, busy_b)[0, 1])
    out["busy_max_over_mean"] = float(busy_a.max() / busy_a.mean())
    out["span_max_over_mean"] = float(span_a.max() / span_a.mean())
    out["span_us"] = {"mean": float(span_a.mean() / 100), "max": float(span_a.max() / 100),
                      "p50": float(np.percentile(span_a, 50) / 100), "p99": float(np.percentile(span_a, 99) / 100)}
    out["start_offset_us"] = {"p50": float(np.percentile(start_a, 50) / 100), "max": float(start_a.max() / 100)}
    out["launch_span_us"] = float((a[:, 17].max() - a[:, 16].min()) / 100)
    uk, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    out["waves_per_simd_hist"] = {int(c): int((cnt == c).sum()) for c in np.unique(cnt)}
    simd_busy = np.bincount(inv, weights=busy_a)
    out["simd_busy_max_over_mean"] = float(simd_busy.max() / simd_busy.mean())
    # does span track busy (slow = more work) or placement (slow = slow partner)?
    out["span_vs_busy_corr"] = float(np.corrcoef(span_a, busy_a)[0, 1])
    partner = np.zeros_like(busy_a)
    for k in range(len(uk)):
        idx = np.nonzero(inv == k)[0]
        for i in idx:
            partner[i] = busy_a[idx[idx != i]].sum()
    out["span_vs_partner_busy_corr"] = float(np.corrcoef(span_a, partner)[0, 1])
    wid = hw & 15
    diffpar = 0
    older_faster = 0
    for k in range(len(uk)):
        idx = np.nonzero(inv == k)[0]
        if len(idx) == 2:
            diffpar += int((wid[idx[0]] & 1) != (wid[idx[1]] & 1))
            first = idx[np.argmin(a[idx, 16])]  # dispatched first
            older_faster += int(span_a[first] <= span_a[idx].max())
    out["pairs_wave_id_parity_differs"] = diffpar / len(uk)
    out["pairs_first_started_is_faster"] = older_faster / len(uk)
    out["wave_id_hist"] = {int(v): int((wid == v).sum()) for v in np.unique(wid)}
    slow = np.argsort(-span_a)[:10]
    out["slowest"] = [{"wave": int(i), "span_us": float(span_a[i] / 100), "busy": int(busy_a[i]),
                       "busy_next": int(busy_b[i]), "partner_busy": int(partner[i]), "xcc": int(xcc[i]),
                       "cu": int(cu[i]), "simd": int(simd[i])} for i in slow]
    print(json.dumps(out, indent=1))
    env.close()


if __name__ == "__main__":
    main()
