"""Parity at BASELINE's full size (65,536 envs) through size-independent
properties: the oracle cannot step 65k envs in test time, so

* shard invariance: any contiguous slice [k, k+m) of the 65k batch evolves
  bit-identically to a separate m-env batch with the same seeds and policy
  offset (the exact property multi-GPU sharding relies on), and that small
  batch is itself checked against the CPU oracle on a sample;
* mask consistency: every env's stored 192-bit mask equals the legal-anchor
  set recomputed on the host from its board and hand;
* determinism: two runs from the same seeds give identical states;
* the multi-rank bench path (2 ranks sharing the card over gloo).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import bb_game as O
from oracle import philox

pytestmark = pytest.mark.gpu

N_FULL = 65536
STEPS = 40
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, offset, steps, cuda):
    from runtime.device_env import DeviceEnvBatch

    env = DeviceEnvBatch(n, seeds=[42 + offset + i for i in range(n)], device=cuda, env_offset=offset)
    env.reset()
    mb = torch.zeros((n, 3), dtype=torch.int64, device=cuda)
    env.obs(mask_bits=mb)
    act = [torch.zeros(n, dtype=torch.int32, device=cuda) for _ in range(2)]
    env.random_actions(mb, act[0], seed=0xB10C, step=0)
    for t in range(steps):
        env.step(act[t & 1], next_action=act[(t + 1) & 1], policy_seed=0xB10C, policy_step=t + 1)
    torch.cuda.synchronize()
    st = env.state()
    env.obs(mask_bits=mb)
    st["mask"] = mb.cpu().numpy().view(np.uint64)
    env.close()
    return st


@pytest.fixture(scope="module")
def full(cuda):
    return _run(N_FULL, 0, STEPS, cuda)


@pytest.mark.parametrize("k", [0, 12345, N_FULL - 300])
def test_shard_invariance(cuda, full, k):
    m = 300
    small = _run(m, k, STEPS, cuda)
    for key, v in small.items():
        assert np.array_equal(full[key][k:k + m], v), key


def test_small_shard_matches_oracle(cuda):
    """The slice batch used above against the CPU oracle (same seeds, the
    same Philox policy on the oracle's own masks)."""
    k, m = 4321, 24
    small = _run(m, k, STEPS, cuda)
    cpu = O.VecEnv(m, seed=42 + k)
    oc, _ = cpu.reset()
    acts = philox.random_policy(oc["action_mask"].astype(bool), 0xB10C, 0, env_offset=k)
    for t in range(STEPS):
        oc, *_ = cpu.step(acts)
        acts = philox.random_policy(oc["action_mask"].astype(bool), 0xB10C, t + 1, env_offset=k)
    ps = cpu.packed_state()
    assert np.array_equal(small["board"], ps["board"])
    for key in ("score", "moves", "lines", "combo", "max_combo", "blocks"):
        assert np.array_equal(small[key].astype(np.int64), ps[key].astype(np.int64)), key


def _anchors_np(piece_bits, boards):
    """Legal anchors of one piece on many boards (host restatement, vectorised)."""
    from game.pieces import PIECE_BITS  # noqa: F401  (table import check)

    cells = [c for c in range(64) if (piece_bits >> c) & 1]
    h = max(c // 8 for c in cells)
    w = max(c % 8 for c in cells)
    out = np.zeros(boards.shape, dtype=np.uint64)
    for r in range(8 - h):
        for c in range(8 - w):
            a = r * 8 + c
            shape = np.uint64(piece_bits << a)
            free = (boards & shape) == 0
            out |= np.where(free, np.uint64(1 << a), np.uint64(0))
    return out


def test_full_size_masks_consistent(full):
    from game.pieces import PIECE_BITS

    bits = [int(b) for b in PIECE_BITS]
    boards = full["board"]
    hand = full["hand"]
    mask = full["mask"]
    for s in range(3):
        ids = (hand >> np.uint32(6 * s)) & np.uint32(63)
        used = ((hand >> np.uint32(18 + s)) & np.uint32(1)).astype(bool)
        exp = np.zeros(boards.shape, dtype=np.uint64)
        for pid in range(37):
            sel = ids == pid
            if sel.any():
                exp[sel] = _anchors_np(bits[pid], boards[sel])
        exp[used] = 0
        assert np.array_equal(mask[:, s], exp), s
    assert (np.bitwise_count(boards) <= 64).all()


def test_full_size_deterministic(cuda, full):
    again = _run(N_FULL, 0, STEPS, cuda)
    for key in full:
        assert np.array_equal(full[key], again[key]), key


def test_bench_two_ranks_shared_gpu(tmp_path):
    env = dict(os.environ, BB_BENCH_SHARE_GPU="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={29900 + os.getpid() % 50}",
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "10", "--warmup", "3", "--envs", "4096",
           "--dp-steps", "0"]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_envs"] == 8192 and d["value"] > 0
    assert d["scaling"] == "weak" and "cpu_baseline" not in d and "dp_update" not in d


def test_bench_gpus_flag_launches_ranks(tmp_path):
    """`python bench.py --gpus 2` with no launcher starts its own two ranks (the driver's plain form) and adds
    the dp_update leg: per-rank optimizer steps with the gradient all-reduce, both precisions (share mode:
    both ranks on cuda:0 over gloo -- the RCCL world is the driver's 8-GPU run)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["BB_BENCH_SHARE_GPU"] = "1"
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "2",
           "--envs", "4096", "--dp-steps", "3", "--dp-warmup", "1"]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_envs"] == 8192
    for prec in ("fp32", "bf16"):
        dp = d["dp_update"][prec]
        assert dp["rccl_world_size"] == 2 and dp["step_ms"] > 0 and dp["local_step_ms"] > 0
        assert dp["ranks_weights_equal"], dp  # the all-reduced updates left both ranks on the same weights
        assert dp["grad_floats"] >= 5_290_113
