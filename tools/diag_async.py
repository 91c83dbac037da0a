"""Diagnostics (not product): per-wave counters of rollout_async_kernel.

Needs a build with -DBB_ASYNC_DIAG=1 (python tools/variants.py build adiag, loaded with
BBVEC_LIB=tools/variants/libbbvec_adiag.so); sets BB_DEBUG_MODE=16.  Reports per env wave:
iterations per step (T plus blocked iterations), cycles per iteration, blocked env-iterations
and iterations that moved no env (and, with -DBB_ASYNC_DIAG=2, the cycles of each phase of an
iteration); per search wave: calls, envs per call, cycles per call, polls, gen_hands_multi phases.
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
    T = int(os.environ.get("T", "128"))
    epw = int(os.environ.get("E", "64"))  # envs per env wave (BB_ASYNC_ENVS)
    ew, sw = int(os.environ.get("EW", str(256 // epw))), int(os.environ.get("SW", "4"))
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
    nwe = (n + epw - 1) // epw
    nws = (n + epw * ew - 1) // (epw * ew) * sw
    soff = 16 * nwe  # the kernel writes the search waves' records (16 words each) from here
    for call in range(4):
        env.rollout(T, act[0], rew, term, next_action=act[1], policy_step0=call * T)
        act.reverse()
        torch.cuda.synchronize()
        env.lib.bb_debug_counters(env.handle, buf.ctypes.data_as(C.c_void_p))
        flat = buf.reshape(-1)
        wex = flat[: 16 * nwe].reshape(-1, 16)
        we = wex[:, :4].astype(np.float64)
        wsx = flat[soff: soff + 16 * nws].reshape(-1, 16).astype(np.float64)
        env_ph = wex[:, 4:12].astype(np.float64).sum(axis=0) / we[:, 0].sum()  # cycles per iteration
        ws = wsx[:, :4]
        ph = wsx[:, 4:10].sum(axis=0) / max(ws[:, 0].sum(), 1)  # gen_hands_multi phase cycles per call
        out.append({
            "call": call, "T": T,
            "env_iters_per_step": round(we[:, 0].mean() / T, 4),
            "env_iters_max": int(we[:, 0].max()),
            "env_cyc_per_iter": round(we[:, 1].sum() / we[:, 0].sum(), 1),
            "env_wave_cyc_mean": round(we[:, 1].mean(), 0),
            "env_wave_cyc_max": int(we[:, 1].max()),
            "blocked_envs_per_iter_per_wave": round(we[:, 2].sum() / we[:, 0].sum(), 3),
            "idle_iters_per_wave": round((wex[:, 3] & 0xFFFFFFFF).astype(np.float64).mean(), 2),
            "idle_cyc_frac": round((wex[:, 3] >> 32).astype(np.float64).sum() / we[:, 1].sum(), 4),
            "env_phase_cyc_per_iter": {k: round(float(v), 0) for k, v in zip(
                ("move_draw", "quick_post", "poll", "philox", "masks", "reward", "outputs_reset", "policy"), env_ph)},
            "search_calls_per_wave": round(ws[:, 0].mean(), 1),
            "envs_per_call": round(ws[:, 1].sum() / max(ws[:, 0].sum(), 1), 2),
            "cyc_per_call": round(ws[:, 2].sum() / max(ws[:, 0].sum(), 1), 0),
            "search_busy_frac": round(ws[:, 2].sum() / (we[:, 1].mean() * len(ws)), 3),
            "polls_per_wave": round(ws[:, 3].mean(), 1),
            # by env-wave index inside the workgroup (wave k's records are claimed k-th by the search lanes):
            # mean cycles, and how often that index is its workgroup's slowest env wave
            "env_wave_cyc_by_index": [round(float(we[k::ew, 1].mean()), 0) for k in range(ew)],
            "slowest_index_share": [round(float(v), 3) for v in np.bincount(
                we[:, 1].reshape(-1, ew).argmax(axis=1), minlength=ew) / max(len(we) // ew, 1)],
            "wg_cyc_max_over_mean": round(float(we[:, 1].reshape(-1, ew).max(axis=1).max() / we[:, 1].mean()), 4),
            "wg_cyc_mean_of_max": round(float(we[:, 1].reshape(-1, ew).max(axis=1).mean()), 0),
            "call_phase_cyc": {k: round(float(v), 0) for k, v in zip(
                ("setup_draws", "anchors_pack", "pass_quick", "pass_exact", "pass_overhead", "resolve"), ph)},
        })
        buf[:] = 0
        env.lib.bb_debug_counters  # counters are overwritten by every launch
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
