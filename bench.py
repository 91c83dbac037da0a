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
    (N > 1: one rank per GPU; run under torch.distributed.run, or plain
     `python bench.py --gpus N`, which starts torch.distributed.run itself as a
     child process before any GPU call and exits with its code.  Envs are
     independent shards, no collective on the data path -> weak scaling.
     After the env timing every rank also runs the `dp_update` leg: PPO
     optimizer steps on its own 2,048-sample minibatches (BASELINE configs 4
     fp32 and 5 bf16, minibatch_scope per_gpu) with the RCCL gradient
     all-reduce of /root/reference/src/agents/ppo.py:395-401's optimizer step,
     timed beside the same step without the collective)

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


def load_valu(n_envs: int, steps_per_launch: int, build_id: str):
    """The rollout kernel's instruction-issue record (its binding resource) from a committed
    rocprofv3 SQ-counter run (profiles/sq_rollout_kernel.json, tools/sq_summary.py --json), or None when it
    was taken on another shape or on a library built from other sources than the loaded one."""
    p = os.path.join(REPO, "profiles", "sq_rollout_kernel.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if int(d.get("n_envs", -1)) != n_envs or int(d.get("steps_per_launch", -1)) != steps_per_launch:
        return None
    if d.get("build_id") != build_id:
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


def load_traffic(n_envs: int, mode: str, steps_per_launch: int, build_id: str):
    """HBM bytes per launch from a committed rocprofv3 PMC run
    (profiles/pmc_step_kernel.json or pmc_rollout_kernel.json, written by
    tools/pmc_traffic.py from two separate --pmc passes, FETCH_SIZE doubled
    per the gfx950 note), or None when it was taken on another shape or on a
    library built from other sources than the loaded one."""
    p = os.path.join(REPO, "profiles", f"pmc_{mode}_kernel.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if (int(d.get("n_envs", -1)) == n_envs and int(d.get("steps_per_launch", 1)) == steps_per_launch
                and d.get("build_id") == build_id):
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` without a launcher: start torch.distributed.run with N ranks of this same
    command line as a child process (nothing here has touched the GPU) and return its exit code."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    print(f"[bench] --gpus {n}: launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=dict(os.environ))


def _dp_minibatches(n: int, dev, seed: int):
    """A rank's synthetic minibatch of n samples: the packed step's six inputs (boards + hand planes,
    192-way masks with at least one legal action, a legal action, old log-prob, advantage, return)."""
    import torch

    g = torch.Generator(device="cpu").manual_seed(seed)
    x = (torch.rand((n, 4, 8, 8), generator=g) < 0.4).float()
    masks = (torch.rand((n, 192), generator=g) < 0.3).float()
    masks[:, 0] = 1.0
    act = torch.multinomial(masks, 1, generator=g).squeeze(1)
    lp = -torch.rand(n, generator=g) * 4.0
    adv = torch.randn(n, generator=g)
    ret = torch.randn(n, generator=g)
    return [t.to(dev) for t in (x, masks, act, lp, adv, ret)]


def dp_update_leg(dev, rank: int, world: int, steps: int, warmup: int, bf16: bool) -> dict:
    """Per-rank PPO optimizer steps of 2,048 samples (train_minibatch: HIP-graph-replayed forward, fused loss,
    backward, gradient all-reduce over the process group -- RCCL on GPUs -- then clip + Adam), timed between
    barriers (max over ranks), and the same step with no collective (a local agent, world forced to 1): the
    difference is the all-reduce's exposed time plus the data-parallel step's own extras.  Plus the full-buffer
    all-reduce alone."""
    import torch
    import torch.distributed as dist

    from agents import ppo as P

    def timed(agent, k, sync_ranks):
        ins = _dp_minibatches(2048, dev, 1000 + rank)
        for _ in range(warmup):
            agent.train_minibatch(*ins)
        if sync_ranks:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            agent.train_minibatch(*ins)
        torch.cuda.synchronize(dev)
        if sync_ranks:
            dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        if sync_ranks:  # max over ranks (gloo-free: the process group's own device for nccl)
            el = el.to(dev) if dist.get_backend() == "nccl" else el
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el.item()) / k * 1e3

    def make_agent():
        torch.manual_seed(0)
        a = P.PPOAgent(P.PPOConfig(batch_size=2048), device=dev, sample_seed=1)
        if bf16:
            a.autocast_dtype = torch.bfloat16
        a.train()
        return a

    # the same step without the collective: world forced to 1 for a local agent (its own graphs)
    P._WORLD_OVERRIDE = 1
    try:
        local_ms = timed(make_agent(), steps, sync_ranks=False)
    finally:
        P._WORLD_OVERRIDE = None
    agent = make_agent()
    P.broadcast_parameters(agent, 0)
    dp_ms = timed(agent, steps, sync_ranks=True)
    flat = agent._flat_grad
    # the full-size collective alone (every gradient float of the model, one buffer)
    for _ in range(3):
        dist.all_reduce(flat)
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(10):
        dist.all_reduce(flat)
    torch.cuda.synchronize(dev)
    ar_ms = (time.perf_counter() - t0) / 10 * 1e3
    # every rank's weights must agree after the data-parallel steps (the all-reduced update is identical)
    w = torch.cat([p.detach().reshape(-1)[:64].double() for p in agent.network.parameters()])
    w_max, w_min = w.clone(), w.clone()
    dist.all_reduce(w_max, op=dist.ReduceOp.MAX)
    dist.all_reduce(w_min, op=dist.ReduceOp.MIN)
    return {
        "workload": ("BASELINE config 5 shape: 131,072 envs per rank's update, bf16 autocast CNN" if bf16 else
                     "BASELINE config 4 shape: default.yaml PPO, fp32 CNN"),
        "minibatch_per_rank": 2048, "scope": "per_gpu (training.minibatch_scope)",
        "dp_overlap": agent.dp_overlap,
        "backend": dist.get_backend(), "rccl_world_size": dist.get_world_size(),
        "steps": steps, "warmup": warmup,
        "step_ms": round(dp_ms, 4), "local_step_ms": round(local_ms, 4),
        # the collective's exposed time plus the data-parallel step's own extras (the flat gradient buffer's
        # zero fill and views, the two backward segments, the average) over the single-rank step
        "dp_minus_local_ms": round(dp_ms - local_ms, 4),
        "allreduce_alone_ms": round(ar_ms, 4), "grad_floats": int(flat.numel()),
        "grad_bytes": int(flat.numel() * 4),
        "allreduce_busbw_gbs": round(2 * (world - 1) / world * flat.numel() * 4 / (ar_ms * 1e-3) / 1e9, 2),
        "ranks_weights_equal": bool(torch.equal(w_max, w_min)),
        "samples_per_s": round(world * 2048 / (dp_ms * 1e-3), 1),
        "optimizer_step": "/root/reference/src/agents/ppo.py:395-401 inside scripts/train.py:173-209",
    }


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
    ap.add_argument("--dp-steps", type=int, default=20,
                    help="N > 1: timed optimizer steps per precision in the dp_update leg (0: no leg)")
    ap.add_argument("--dp-warmup", type=int, default=5)
    ap.add_argument("--dp-precision", choices=("fp32", "bf16", "both"), default="both",
                    help="dp_update leg: config 4's fp32 CNN, config 5's bf16 autocast CNN, or both")
    ap.add_argument("--dp-timeout", type=float, default=300.0,
                    help="dp_update leg watchdog (s): on expiry rank 0 prints the line with the error")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: launch N ranks for --gpus N", file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist

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
    for e, _, _, _ in shards:  # the env shards' memory is not needed by the update leg
        e.close()
    shards = []

    def line(dp_block):
        """The bench line (rank 0 prints it)."""
        algo_bytes = ALGO_BYTES_PER_ENV_STEP * n * per_launch
        achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
        bid = L.build_id()
        traffic = load_traffic(n, args.mode, per_launch, bid)
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
            "build_id": bid,
        }
        if args.mode == "rollout":
            # the binding resource is instruction issue, not bytes: the committed SQ counters
            out["roofline"]["valu"] = load_valu(n, T, bid)
        if dp_block is not None:
            out["dp_update"] = dp_block
        return out

    dp = None
    if world > 1 and args.dp_steps > 0:
        # the env line is already measured: a dp_update leg that fails or hangs (a collective that never
        # completes) must not cost it.  A watchdog per rank prints rank 0's line with the error and ends
        # every rank with status 0 after --dp-timeout seconds; an exception is recorded likewise.
        import threading

        dp = {}

        def expire():
            if rank == 0:
                dp["error"] = f"dp_update leg timed out after {args.dp_timeout:.0f} s"
                print(json.dumps(line(dp)), flush=True)
            print(f"[bench] rank {rank}: dp_update watchdog fired", file=sys.stderr, flush=True)
            os._exit(0)

        dog = threading.Timer(args.dp_timeout, expire)
        dog.daemon = True
        dog.start()
        try:
            for prec in (("fp32", "bf16") if args.dp_precision == "both" else (args.dp_precision,)):
                dp[prec] = dp_update_leg(dev, rank, world, args.dp_steps, args.dp_warmup, prec == "bf16")
        except Exception as exc:  # noqa: BLE001 -- reported in the line, never lost
            dp["error"] = f"{type(exc).__name__}: {exc}"[:500]
            print(f"[bench] rank {rank}: dp_update leg failed: {dp['error']}", file=sys.stderr, flush=True)
        dog.cancel()
    if rank == 0:
        out = line(dp)
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(args.cpu_seconds)
            out["cpu_baseline"] = cb
            if not args.no_native_baseline:
                out["cpu_baseline_native"] = cpu_baseline_native(args.native_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
