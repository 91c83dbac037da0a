"""Diagnostics (not product): where a single bb_step launch (T = 1) spends its time in steady state.

Needs the diag3 build (BBVEC_LIB=tools/variants/libbbvec_diag3.so).  Envs are first advanced WARM steps with
a 128-step rollout so the boards are mid-game, then CALLS single-step launches are recorded.  Per launch:
the slowest wave, the 2nd / 4th / 16th slowest, the mean; the slowest wave's share of search cycles; how
many workgroups hold a wave slower than 2x / 4x the mean; the realtime span of the waves (100 MHz stamps).
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
    n = int(os.environ.get("N", "65536"))
    warm = int(os.environ.get("WARM", "256"))
    calls = int(os.environ.get("CALLS", "64"))
    epw, wpg = 32, 8
    dev = torch.device("cuda", 0)
    env = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device=dev)
    env.reset()
    mb = torch.zeros((n, 3), dtype=torch.int64, device=dev)
    env.obs(mask_bits=mb)
    act = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
    env.random_actions(mb, act[0], step=0)
    T = 128
    rew = torch.zeros((T, n), dtype=torch.float32, device=dev)
    term = torch.zeros((T, n), dtype=torch.uint8, device=dev)
    for k in range(warm // T):
        env.rollout(T, act[0], rew, term, next_action=act[1], policy_step0=k * T)
        act.reverse()
    step0 = (warm // T) * T
    buf = np.zeros((n, 4), dtype=np.uint64)  # bb_debug_counters copies n * 32 bytes
    rows = []
    for c in range(calls):
        env.rollout(1, act[0], rew[:1], term[:1], next_action=act[1], policy_step0=step0 + c)
        act.reverse()
        torch.cuda.synchronize()
        env.lib.bb_debug_counters(env.handle, buf.ctypes.data_as(C.c_void_p))
        w = buf.reshape(-1)[: (n // epw) * 18].reshape(-1, 18)
        tot = (w[:, 0] + w[:, 1] + w[:, 2]).astype(np.float64)
        srt = np.sort(tot)[::-1]
        mean = float(tot.mean())
        wg = tot.reshape(-1, wpg)
        t0 = w[:, 16].astype(np.int64)
        t1 = w[:, 17].astype(np.int64)
        k = int(np.argmax(tot))
        rows.append({
            "max": int(srt[0]), "2nd": int(srt[1]), "4th": int(srt[3]), "16th": int(srt[15]), "mean": round(mean),
            "max_search_frac": round(float(w[k, 1]) / max(srt[0], 1), 3),
            "max_parked": int(w[k, 3] & np.uint64(0xFFFFFFFF)),
            "max_phases": {q: int(w[k, 9 + j]) for j, q in enumerate(
                ("setup_draw", "anchors_scan", "pass_quick", "pass_exact", "pass_flags", "resolve"))} | {
                "move_quick": int(w[k, 0]), "search": int(w[k, 1]), "finalize": int(w[k, 2])},
            "wg_gt2x": int((wg.max(axis=1) > 2 * mean).sum()), "wg_gt4x": int((wg.max(axis=1) > 4 * mean).sum()),
            "wg_sum_over_max": round(float(np.median(wg.sum(axis=1) / wg.max(axis=1))), 2),
            "span_us": round(float(t1.max() - t0.min()) / 100.0, 2),
            "wave_start_spread_us": round(float(t0.max() - t0.min()) / 100.0, 2),
        })
    keys = [k for k in rows[0] if k not in ("max_parked", "max_phases")]
    summ = {k: round(float(np.mean([r[k] for r in rows])), 2) for k in keys}
    summ["max_p50"] = float(np.median([r["max"] for r in rows]))
    summ["max_p10"] = float(np.percentile([r["max"] for r in rows], 10))
    print(json.dumps({"n": n, "warm": warm, "calls": calls, "mean_over_calls": summ, "calls_detail": rows[:16]},
                     indent=1))
    env.close()


if __name__ == "__main__":
    main()
