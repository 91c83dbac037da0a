"""Diagnostics (not product): per-wave phase cycles of bb_rollout.

Needs a build with -DBB_ROLL_DIAG=3 (tools/build_variant.sh diag3 -DBB_ROLL_DIAG=3,
loaded with BBVEC_LIB=...) and BB_DEBUG_MODE=16.  Reports, summed over waves
and steps: move + in-lane quick test, wave searches, finalize; the number of
searches, attempts, passes, slow passes and the quick / disjoint / line
cycles inside the searches.
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
    T = int(os.environ.get("T", "200"))
    epw = int(os.environ.get("EPW", "32"))
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
    out = []
    for call in range(3):  # the first call covers the synchronised start of every episode
        env.rollout(T, act[0], rew, term, next_action=act[1], policy_step0=call * T)
        act.reverse()
        torch.cuda.synchronize()
        env.lib.bb_debug_counters(env.handle, buf.ctypes.data_as(C.c_void_p))
        w = buf.reshape(-1)[: (n // epw) * 18].reshape(-1, 18)
        lo = lambda v: float((v & np.uint64(0xFFFFFFFF)).astype(np.float64).sum())  # noqa: E731
        hi = lambda v: float((v >> np.uint64(32)).astype(np.float64).sum())  # noqa: E731
        tot = w.sum(axis=0).astype(np.float64)
        for c in (3, 4, 6):
            tot[c] = lo(w[:, c])
        waves = w.shape[0]
        per = lambda x: round(x / waves / T, 1)  # noqa: E731  cycles per wave per step
        out.append({
            "call": call, "waves": waves, "T": T,
            "cyc_per_wave_step": {"move_quick": per(tot[0]), "search": per(tot[1]), "finalize": per(tot[2])},
            "multi_search_per_wave_step": {k: per(tot[9 + q]) for q, k in enumerate(
                ("setup_draw", "anchors_scan", "pass_quick", "pass_exact", "pass_flags", "resolve"))},
            "max_wave_total": int((w[:, 0] + w[:, 1] + w[:, 2]).max()),
            "mean_wave_total": float((w[:, 0] + w[:, 1] + w[:, 2]).astype(np.float64).mean()),
            "searches_per_wave_step": round(tot[3] / waves / T, 3),
            "attempts_per_search": round(tot[4] / max(tot[3], 1), 2),
            "passes_per_search": round(lo(w[:, 5]) / max(tot[3], 1), 2),
            "slow_passes_per_search": round(hi(w[:, 5]) / max(tot[3], 1), 2),
            "slots_per_pass": round(hi(w[:, 6]) / max(lo(w[:, 5]), 1), 2),
            "undecided_slots_per_search": round(hi(w[:, 3]) / max(tot[3], 1), 2),
            "frac_first_attempt": round(hi(w[:, 4]) / max(tot[3], 1), 3),
            "frac_first_attempt_quick": round(float(w[:, 8].astype(np.float64).sum()) / max(tot[3], 1), 3),
            "cyc_per_search": {"all": round(tot[1] / max(tot[3], 1)), "quick": round(tot[6] / max(tot[3], 1)),
                               "disjoint": round(lo(w[:, 7]) / max(tot[3], 1)),
                               "line": round(hi(w[:, 7]) / max(tot[3], 1))},
        })
    print(json.dumps(out, indent=1))
    env.close()


if __name__ == "__main__":
    main()
