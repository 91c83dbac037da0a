"""Bit-exact parity at BASELINE's full size against the C oracle.

The C oracle (oracle/bb_oracle.c: cell grids, the reference's recursive DFS,
numpy-exact PCG64; pinned by tests/test_c_oracle.py against the seed-42
golden, numpy and the Python oracle) steps all 65,536 envs on the host, so the
HIP kernels are compared output for output at the bench shape itself:

* bb_rollout, two launches of T = 128 (the bench step), env i seeded 42 + i;
* a shard of an 8-GPU run (global offset 3 x 65,536) with half of its envs
  unseeded (seed_value None: the stream continues across resets);
* bb_step (step + escalate kernels) for 64 steps, the VectorizedBlockBlastEnv
  drop-in path;
* a custom reward config without auto-reset (single-env semantics).

Every per-step output (f32 reward bits, terminated, lines cleared, applied
action, post-step 192-bit mask) and the final per-env state are compared.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import c_oracle as CO

pytestmark = pytest.mark.gpu

SEED = 0xB10C
N_FULL = 65536
T = 128


def _gpu_env(n, offset, cuda, unseeded=None, reward_config=None, autoreset=True):
    from runtime.device_env import DeviceEnvBatch

    seeds = np.arange(42 + offset, 42 + offset + n, dtype=np.uint64)
    env = DeviceEnvBatch(n, seeds=[int(s) for s in seeds], device=cuda, env_offset=offset,
                         reward_config=reward_config, autoreset=autoreset)
    if unseeded is not None:  # raw PCG words = default_rng(seed) words, seed_value None
        has = np.where(unseeded, 0, 1).astype(np.uint8)
        raw = np.array([CO.pcg64_seed(int(s)) for s in seeds], dtype=np.uint64)
        assert env.lib.bb_seed(env.handle, seeds.ctypes.data_as(C.c_void_p), has.ctypes.data_as(C.c_void_p),
                               raw.ctypes.data_as(C.c_void_p)) == 0
    env.reset()
    return env, seeds


def _cpu_env(seeds, unseeded=None, reward_config=None, autoreset=True):
    c = CO.CVecEnv(seeds, reward_config=reward_config, autoreset=autoreset,
                   has_seed=None if unseeded is None else np.where(unseeded, 0, 1))
    c.reset()
    return c


def _same_state(g, c):
    gs, cs = g.state(), c.state()
    for k in ("board", "hand", "score", "combo", "max_combo", "moves", "lines", "blocks", "prev_holes",
              "prev_center"):
        assert np.array_equal(gs[k], cs[k]), f"state {k}"
    assert np.array_equal(gs["rng"][:, :2], cs["rng"][:, :2]), "pcg state"
    has = ((cs["hand"] >> np.uint32(22)) & np.uint32(1)).astype(bool)
    assert np.array_equal(gs["rng"][has, 2], cs["rng"][has, 2]), "pcg uinteger"
    return cs


def _rollout_vs_oracle(cuda, n, offset, launches, unseeded=None):
    env, seeds = _gpu_env(n, offset, cuda, unseeded)
    cpu = _cpu_env(seeds, unseeded)
    cs = _same_state(env, cpu)
    a0 = cpu.random_actions(cs["mask"], SEED, 0, env_offset=offset)
    a = torch.from_numpy(a0).to(cuda)
    nxt = torch.zeros_like(a)
    rew = torch.zeros((T, n), dtype=torch.float32, device=cuda)
    term = torch.zeros((T, n), dtype=torch.uint8, device=cuda)
    lines = torch.zeros((T, n), dtype=torch.uint8, device=cuda)
    acts = torch.zeros((T, n), dtype=torch.int32, device=cuda)
    masks = torch.zeros((T, n, 3), dtype=torch.int64, device=cuda)
    ca = a0
    terminations = 0
    for k in range(launches):
        env.rollout(T, a, rew, term, lines=lines, actions_out=acts, mask_out=masks, next_action=nxt,
                    policy_seed=SEED, policy_step0=k * T)
        a, nxt = nxt, a
        ref = cpu.rollout(T, ca, policy_seed=SEED, policy_step0=k * T, env_offset=offset)
        ca = ref["next_action"]
        torch.cuda.synchronize()
        assert np.array_equal(rew.cpu().numpy().view(np.uint32), ref["reward"].view(np.uint32)), f"reward {k}"
        assert np.array_equal(term.cpu().numpy(), ref["terminated"]), f"terminated {k}"
        assert np.array_equal(lines.cpu().numpy(), ref["lines"]), f"lines {k}"
        assert np.array_equal(acts.cpu().numpy(), ref["actions"]), f"actions {k}"
        assert np.array_equal(masks.cpu().numpy().view(np.uint64), ref["mask"]), f"mask {k}"
        assert np.array_equal(a.cpu().numpy(), ca), f"next action {k}"
        terminations += int(ref["terminated"].sum())
    _same_state(env, cpu)
    env.close()
    return terminations


def test_full_size_rollout_matches_c_oracle(cuda):
    """The bench workload itself: 65,536 envs, two bb_rollout launches of 128 steps."""
    assert _rollout_vs_oracle(cuda, N_FULL, 0, launches=2) > 1000  # many episodes end and re-seed


def test_full_size_shard_unseeded_matches_c_oracle(cuda):
    """Rank 3 of an 8-GPU run (global env offset 3 x 65,536), every other env
    unseeded (seed_value None)."""
    unseeded = (np.arange(N_FULL) % 2) == 1
    assert _rollout_vs_oracle(cuda, N_FULL, 3 * N_FULL, launches=1, unseeded=unseeded) > 0


@pytest.mark.parametrize("kernels", ["1", "2"])
def test_full_size_step_path_matches_c_oracle(cuda, kernels, monkeypatch):
    """bb_step at 65,536 envs, 64 steps, the VectorizedBlockBlastEnv.step
    drop-in path: fused (rollout kernel at T = 1, default) and step_kernel +
    escalate_kernel (BB_STEP_KERNELS=2)."""
    monkeypatch.setenv("BB_STEP_KERNELS", kernels)
    n, steps = N_FULL, 64
    env, seeds = _gpu_env(n, 0, cuda)
    cpu = _cpu_env(seeds)
    cs = _same_state(env, cpu)
    a = cpu.random_actions(cs["mask"], SEED, 0)
    mb = torch.zeros((n, 3), dtype=torch.int64, device=cuda)
    nxt = torch.zeros(n, dtype=torch.int32, device=cuda)
    for t in range(steps):
        ga = torch.from_numpy(a).to(cuda)
        env.step(ga, want_lines=True, want_f64=True, next_action=nxt, policy_seed=SEED, policy_step=t + 1,
                 mask_out=mb)
        o = cpu.step(a)
        torch.cuda.synchronize()
        assert np.array_equal(env.reward_f64.cpu().numpy(), o["reward_f64"]), t
        assert np.array_equal(env.terminated.cpu().numpy(), o["terminated"]), t
        assert np.array_equal(env.lines.cpu().numpy(), o["lines"]), t
        assert np.array_equal(mb.cpu().numpy().view(np.uint64), o["mask"]), t
        a = cpu.random_actions(o["mask"], SEED, t + 1)
        assert np.array_equal(nxt.cpu().numpy(), a), t
    _same_state(env, cpu)
    env.close()


def test_custom_rewards_no_autoreset_matches_c_oracle(cuda):
    """Single-env semantics (no auto-reset) with a custom reward config, a
    random mix of legal and illegal actions, 16,384 envs x 150 steps."""
    n, steps = 16384, 150
    rw = {"line_clear_base": 2.5, "block_placed": 0.03, "game_over_penalty": -3.0, "hole_penalty": -0.25,
          "center_bonus": 0.7, "combo_multiplier_bonus": 1.25, "survival_bonus": 0.0625}
    env, seeds = _gpu_env(n, 0, cuda, reward_config=rw, autoreset=False)
    cpu = _cpu_env(seeds, reward_config=rw, autoreset=False)
    cs = _same_state(env, cpu)
    rng = np.random.default_rng(5)
    mask = cs["mask"]
    for t in range(steps):
        a = cpu.random_actions(mask, SEED, t)
        bad = rng.random(n) < 0.1
        a[bad] = rng.integers(-2, 200, size=int(bad.sum()))
        env.step(torch.from_numpy(a).to(cuda), want_f64=True)
        o = cpu.step(a)
        mask = o["mask"]
        torch.cuda.synchronize()
        assert np.array_equal(env.reward_f64.cpu().numpy(), o["reward_f64"]), t
        assert np.array_equal(env.terminated.cpu().numpy(), o["terminated"]), t
    st = _same_state(env, cpu)
    assert ((st["hand"] >> np.uint32(21)) & np.uint32(1)).any()  # games ended and stayed over
    env.close()
