#!/usr/bin/env python
"""Benchmark: env-steps/sec of the gfx950 vec-env (BASELINE.json metric).

Default workload (BASELINE config 2, one GPU): 65,536 envs per GPU, env i
seeded 42 + global index, HIP bitboard step + action mask + in-kernel
auto-reset, actions from the synthetic random policy (Philox, fused into the
kernel).  A bench "step" is one pass of the hot path over one batch:
  --mode rollout (default): one bb_rollout launch = T = 128 env-steps (the
      reference's PPO horizon, scripts/train.py:173-203 / config n_steps) of
      every env, the env state held in registers between its T steps;
  --mode step: one bb_step call = one env-step of every env, the drop-in path
      under VectorizedBlockBlastEnv.step (one launch of the rollout kernel at
      T = 1; BB_STEP_KERNELS=2 selects the step + escalate kernel pair).
Both produce identical trajectories (tests/test_gpu_rollout.py).  `value`
counts env-steps (envs x T x K in rollout mode, envs x K in step mode) over
the timed wall time.

    python bench.py --gpus N --steps K --warmup W [--mode rollout|step]
    (N > 1: launched by torch.distributed.run, one rank per GPU; envs are
     independent shards, no collective on the data path -> weak scaling)

Prints ONE JSON line on rank 0.  `roofline` prices the dominant kernel
against HBM with the algorithmic bytes of SURVEY.md 8(d) (194 B per env-step)
x the env-steps of one launch, over its average launch duration measured here
with HIP events on the launch stream (the rocprofv3 kernel-trace average
agrees, profiles/); `cpu_baseline` times the CPU port of the reference's
64-env vectorised path (oracle/bb_game.py, one core) on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

ALGO_BYTES_PER_ENV_STEP = 194  # 2x80 B state + 4 action + 24 mask + 4 reward + 1 term + 1 lines
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
POLICY_SEED = 0xB10C


def host_facts() -> dict:
    """the host the CPU baselines ran on -- CPU model, visible cores, torch threads."""
    import torch

    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "torch_threads": torch.get_num_threads(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def load_valu(n_envs: int, steps_per_launch: int):
    """The rollout kernel's instruction-issue record (its binding resource) from a committed
    rocprofv3 SQ-counter run (profiles/sq_rollout_kernel.json, tools/sq_summary.py --json), or None when it
    was taken on another shape."""
    p = os.path.join(REPO, "profiles", "sq_rollout_kernel.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if int(d.get("n_envs", -1)) != n_envs or int(d.get("steps_per_launch", -1)) != steps_per_launch:
        return None
    keys = ("valu_insts_per_launch", "valu_insts_per_env_step", "wave_cycles_per_env_step",
            "cycles_per_valu_per_simd", "issue_floor_cycles", "issue_frac", "profiled_ms", "build_id")
    out = {k: d[k] for k in keys if k in d}
    out["source"] = "profiles/sq_rollout_kernel.json (rocprofv3 --pmc SQ_INSTS_VALU, SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE)"
    return out


def cpu_baseline(seconds: float = 12.0) -> dict:
    """Reference path on the host: 64 envs stepped sequentially by the CPU
    port of src/environment/wrappers.py (cell loops like the reference), with
    random legal actions.  Bounded to ~`seconds` of CPU work."""
    import numpy as np

    from oracle import bb_game as O

    n = 64
    vec = O.VecEnv(n, seed=42)
    obs, _ = vec.reset()
    rng = np.random.default_rng(0)
    steps = 0
    t0 = time.perf_counter()
    while True:
        masks = obs["action_mask"].astype(bool)
        acts = np.array([rng.choice(np.nonzero(m)[0]) for m in masks])
        obs, *_ = vec.step(acts)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {
        "value": round(n * steps / el, 2),
        "unit": "env-steps/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{n} envs x {steps} vec steps ({n * steps} env-steps, {el:.1f}s), random legal actions, "
                  "CPU port of wrappers.py/block_blast_env.py/engine.py (oracle/bb_game.py), 1 Python thread",
        "reference_loop": "/root/reference/src/environment/wrappers.py:75-116 (sequential BlockBlastEnv.step loop)",
        **host_facts(),
    }


def cpu_baseline_native(seconds: float = 8.0, n: int = 65536, T: int = 16) -> dict:
    """The same workload on the host's cores through the C-ABI's host backend
    (libbbvec_host.so, csrc/bb_host.cpp: bitboard step + mask + auto-reset +
    Philox policy, one env per OpenMP thread iteration) -- the reference's
    algorithm as native multi-threaded code, beside the port's 1-thread
    number.  Bounded to ~`seconds`."""
    import torch

    from runtime import lib as L
    from runtime.device_env import DeviceEnvBatch

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    e = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device="cpu")
    e.reset()
    mb = torch.zeros((n, 3), dtype=torch.int64)
    e.obs(mask_bits=mb)
    a = [torch.zeros(n, dtype=torch.int32), torch.zeros(n, dtype=torch.int32)]
    e.random_actions(mb, a[0], seed=POLICY_SEED, step=0)
    rew = torch.zeros((T, n), dtype=torch.float32)
    term = torch.zeros((T, n), dtype=torch.uint8)
    launches = 0
    t0 = time.perf_counter()
    while True:
        e.rollout(T, a[0], rew, term, next_action=a[1], policy_seed=POLICY_SEED, policy_step0=launches * T)
        a.reverse()
        launches += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    e.close()
    return {
        "value": round(n * T * launches / el, 1),
        "unit": "env-steps/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n} envs x {T * launches} env-steps ({launches} bb_rollout calls of T={T}, {el:.1f}s), fused "
                  f"random legal-action policy, host backend libbbvec_host.so (C++ bitboards, OpenMP, "
                  f"{threads} threads)",
        "reference_loop": "/root/reference/src/environment/wrappers.py:75-116, restated natively over all envs",
        "build_id": L.build_id(host=True),
        **host_facts(),
    }


def load_traffic(n_envs: int, mode: str, steps_per_launch: int):
    """HBM bytes per launch from a committed rocprofv3 PMC run
    (profiles/pmc_step_kernel.json or pmc_rollout_kernel.json, written by
    tools/pmc_traffic.py from two separate --pmc passes, FETCH_SIZE doubled
    per the gfx950 note), or None when it was taken on another shape."""
    p = os.path.join(REPO, "profiles", f"pmc_{mode}_kernel.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if int(d.get("n_envs", -1)) == n_envs and int(d.get("steps_per_launch", 1)) == steps_per_launch:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 timed launches after 20 warm-up launches (0.13 s of kernels): the first launches after the reset run the
    # young-episode mix and read ~3.5% under the steady state of a PPO run (20 after 5: 1.337e10; 20 after 100:
    # 1.380e10; 200 after 20 or 100: 1.390e10; 1,280 after 128: 1.391e10, profiles/r05/r05wu_*)
    ap.add_argument("--steps", type=int, default=200,
                    help="timed bench steps: bb_rollout launches of T env-steps (rollout) or bb_step launches (step)")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-native-baseline", action="store_true")
    ap.add_argument("--native-seconds", type=float, default=8.0)
    ap.add_argument("--mode", choices=("rollout", "step"), default="rollout",
                    help="rollout: bb_rollout, T fused env-steps per launch (default); step: one bb_step per env-step")
    ap.add_argument("--shards", type=int, default=1,
                    help="split the envs into this many handles, one HIP stream each")
    ap.add_argument("--rollout-len", type=int, default=128,
                    help="T, env-steps per bb_rollout launch (default 128 = the reference's PPO horizon n_steps)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BB_BENCH_SHARE_GPU=1 (tests only): every rank on cuda:0 over gloo, to
    # exercise the multi-rank path on a one-GPU box; the numbers are not a bench
    share = os.environ.get("BB_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from runtime import lib as L
    from runtime.device_env import DeviceEnvBatch

    n = args.envs
    offset = rank * n
    S = max(1, args.shards)
    assert n % S == 0
    ns = n // S
    T = max(1, args.rollout_len)
    shards = []  # (env batch, stream, action double buffer, per-step outputs of one launch)
    for k in range(S):
        off = offset + k * ns
        e = DeviceEnvBatch(ns, seeds=[42 + off + i for i in range(ns)], device=dev, env_offset=off)
        e.reset()
        mb = torch.zeros((ns, 3), dtype=torch.int64, device=dev)
        e.obs(mask_bits=mb)
        a = [torch.zeros(ns, dtype=torch.int32, device=dev), torch.zeros(ns, dtype=torch.int32, device=dev)]
        e.random_actions(mb, a[0], seed=POLICY_SEED, step=0)
        outs = None
        if args.mode == "rollout":  # [T][N] (rewritten by every launch)
            outs = (torch.zeros((T, ns), dtype=torch.float32, device=dev),
                    torch.zeros((T, ns), dtype=torch.uint8, device=dev),
                    torch.zeros((T, ns), dtype=torch.uint8, device=dev),
                    torch.zeros((T, ns), dtype=torch.int32, device=dev),
                    torch.zeros((T, ns, 3), dtype=torch.int64, device=dev))
        shards.append((e, torch.cuda.Stream(dev) if S > 1 else torch.cuda.current_stream(dev), a, outs))
    step_idx = [0]
    # diagnostics only, never the bench line's contract: the launch without the lines / action / mask outputs,
    # to price the scattered [step][env] stores of the async rollout
    diag_min_out = os.environ.get("BB_BENCH_MIN_OUTPUTS") == "1"

    def one_step(k=1):
        """k bench steps: k bb_step launches (step mode) or k bb_rollout launches of T env-steps each."""
        t = step_idx[0]
        cur = torch.cuda.current_stream(dev)
        if S > 1:
            for _, st, _, _ in shards:
                st.wait_stream(cur)
        for j in range(k):  # the action double-buffer flips once per launch
            for e, st, a, outs in shards:
                with torch.cuda.stream(st):
                    if args.mode == "step":
                        e.step(a[0], next_action=a[1], policy_seed=POLICY_SEED, policy_step=t + j + 1)
                    else:
                        o_rew, o_term, o_lines, o_act, o_mask = outs
                        if diag_min_out:  # diagnostics only (BB_BENCH_MIN_OUTPUTS=1): reward + terminated
                            o_lines = o_act = o_mask = None
                        e.rollout(T, a[0], o_rew, o_term, lines=o_lines, actions_out=o_act, mask_out=o_mask,
                                  next_action=a[1], policy_seed=POLICY_SEED, policy_step0=t + j * T)
                a.reverse()
        if S > 1:
            for _, st, _, _ in shards:
                cur.wait_stream(st)
        step_idx[0] = t + k * (1 if args.mode == "step" else T)

    one_step(args.warmup)

    # HIP events on the launch stream (torch's current stream) bracket the
    # timed region; no event between steps (each timing event is a queue
    # barrier with a cache flush that would stall the back-to-back launches)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record()
    one_step(args.steps)
    ev1.record()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # average launch (= one bench step): bb_step (both kernels + their gap) or one T-step bb_rollout
    per_launch = 1 if args.mode == "step" else T
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        t = torch.tensor([el, kern_ms], dtype=torch.float64, device="cpu" if share else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern_ms = float(t[0]), float(t[1])

    # sanity: every sampled action was legal -> no -10 rewards in the last step
    for e, _, _, outs in shards:
        last_rew = e.reward if args.mode == "step" else outs[0]
        assert bool((last_rew != -10.0).all()), "random policy produced an illegal action"

    total_env_steps = n * world * args.steps * per_launch
    value = total_env_steps / el
    if rank == 0:
        algo_bytes = ALGO_BYTES_PER_ENV_STEP * n * per_launch
        achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
        traffic = load_traffic(n, args.mode, per_launch)
        out = {
            "metric": "env-steps/sec (whole node) at 64k parallel envs, 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: numpy-exact PCG64 piece streams (env i seed 42+i), Philox random legal-action policy",
            "config": {
                "workload": "BASELINE config 2: 65,536 envs per MI355X, HIP bitboard step + action mask + "
                            "auto-reset, random policy (env throughput)",
                "mode": args.mode if args.mode == "step" else f"rollout T={T}",
                "bench_step": ("one bb_step launch = 1 env-step of every env" if args.mode == "step" else
                               f"one bb_rollout launch = {T} env-steps of every env (the PPO horizon)"),
                "env_steps_per_bench_step": n * world * per_launch,
                "envs_per_gpu": n,
                "global_envs": n * world,
                "parallelism": f"env shards x{world} (no data-path collective)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "kernel": (("bb_step = bb::step_kernel + bb::escalate_kernel (BB_STEP_KERNELS=2)"
                            if os.environ.get("BB_STEP_KERNELS") == "2" else
                            "bb_step = one bb::step_fused_kernel<true> launch") if args.mode == "step" else
                           f"bb_rollout = bb::rollout_async_kernel (env waves + search waves), {T} env-steps "
                           f"of every env per launch"),
                "env_steps_per_launch": n * per_launch,
                "kernel_avg_ms": round(kern_ms, 5),
                "algo_bytes_per_launch": algo_bytes,
            },
            "build_id": L.build_id(),
        }
        if args.mode == "rollout":
            # the binding resource is instruction issue, not bytes: the committed SQ counters
            out["roofline"]["valu"] = load_valu(n, T)
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(args.cpu_seconds)
            out["cpu_baseline"] = cb
            if not args.no_native_baseline:
                out["cpu_baseline_native"] = cpu_baseline_native(args.native_seconds)
        print(json.dumps(out), flush=True)
    for e, _, _, _ in shards:
        e.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
