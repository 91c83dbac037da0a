"""GPU parity: the gfx950 vec-env (through the C-ABI) vs the CPU oracle.

Bit-exact on every step, on both bb_step paths (BB_STEP_KERNELS=1: one launch
of the rollout kernel at T = 1, the default; 2: step_kernel + escalate_kernel):
observations (board / piece planes / int8 mask),
f32 rewards, terminated flags, info dicts (incl. last_move, terminal
observation, final_score) and the full packed state.  Actions mix legal moves
with illegal ones (used slot, collision, off-board, out-of-range ints) so the
invalid-action path (block_blast_env.py:240-245) is exercised too.
"""
import numpy as np
import pytest
import torch

from oracle import bb_game as O
from oracle import philox

pytestmark = pytest.mark.gpu


def _actions(rng, masks, p_invalid):
    out = np.zeros(len(masks), dtype=np.int64)
    for i, m in enumerate(masks):
        valid = np.nonzero(m)[0]
        if rng.random() < p_invalid or valid.size == 0:
            out[i] = int(rng.choice([-7, -1, 192, 200, 10 ** 6, int(rng.integers(0, 192))]))
        else:
            out[i] = int(rng.choice(valid))
    return out


def _cmp_info(gi, ci, where):
    assert set(gi.keys()) == set(ci.keys()), where
    for k, v in ci.items():
        if k == "terminal_observation":
            for kk in ("board", "pieces", "action_mask"):
                assert np.array_equal(gi[k][kk], v[kk]), (where, kk)
        else:
            assert gi[k] == v and type(gi[k]) == type(v), (where, k, gi[k], v)


def _run_parity(n, steps, seed, p_invalid, reward_config=None, act_seed=0):
    from environment.wrappers import VectorizedBlockBlastEnv

    gpu = VectorizedBlockBlastEnv(n, seed=seed, reward_config=reward_config, device="cuda:0")
    cpu = O.VecEnv(n, seed=seed, reward_config=reward_config)
    og, ig = gpu.reset()
    oc, ic = cpu.reset()
    assert len(ig) == n
    rng = np.random.default_rng(act_seed)
    terms = 0
    for t in range(steps):
        for k in ("board", "pieces", "action_mask"):
            assert og[k].dtype == oc[k].dtype and np.array_equal(og[k], oc[k]), (t, k)
        acts = _actions(rng, oc["action_mask"], p_invalid)
        og, rg, tg, trg, ig = gpu.step(acts)
        oc, rc, tc, trc, ic = cpu.step(acts)
        assert rg.dtype == np.float32 and np.array_equal(rg.view(np.uint32), rc.view(np.uint32)), t
        assert np.array_equal(tg, tc) and not trg.any(), t
        terms += int(tc.sum())
        for i in range(n):
            _cmp_info(ig[i], ic[i], (t, i))
    st = gpu.dev.state()
    ps = cpu.packed_state()
    assert np.array_equal(st["board"], ps["board"])
    ids = np.stack([(st["hand"] >> (6 * s)) & 63 for s in range(3)], 1)
    used = np.stack([(st["hand"] >> (18 + s)) & 1 for s in range(3)], 1).astype(bool)
    assert np.array_equal(ids, ps["hand"]) and np.array_equal(used, ps["used"])
    for k in ("score", "moves", "lines", "combo", "max_combo", "blocks"):
        assert np.array_equal(st[k].astype(np.int64), ps[k].astype(np.int64)), k
    gpu.close()
    return terms


@pytest.mark.parametrize("kernels", ["1", "2"])
def test_vec_env_bit_exact_default_rewards(cuda, kernels, monkeypatch):
    monkeypatch.setenv("BB_STEP_KERNELS", kernels)  # 1: fused (rollout kernel, T = 1); 2: step + escalate
    terms = _run_parity(n=96, steps=160, seed=42, p_invalid=0.1)
    assert terms > 50  # auto-reset path exercised many times


@pytest.mark.parametrize("kernels", ["1", "2"])
def test_vec_env_bit_exact_custom_rewards(cuda, kernels, monkeypatch):
    monkeypatch.setenv("BB_STEP_KERNELS", kernels)  # 1: fused (rollout kernel, T = 1); 2: step + escalate
    rc = {"line_clear_base": 100.0, "block_placed": 1.0, "game_over_penalty": -500.0, "hole_penalty": -0.3,
          "center_bonus": 0.7, "combo_multiplier_bonus": 3.25}
    _run_parity(n=64, steps=120, seed=7, p_invalid=0.05, reward_config=rc, act_seed=3)


@pytest.mark.parametrize("budget", ["0", "1", "16", "64", "1000000000", "q1", "q3", "q6"])
def test_vec_env_solver_paths(cuda, monkeypatch, budget):
    """Budget 0 sends every hand search to the wave-cooperative escalation
    kernel, 1 / 16 / 64 escalate after a partial in-lane search, a huge budget
    keeps every search inside its lane, qK tests K fixed slots in-lane.  All
    must reproduce the oracle bit for bit."""
    if budget.startswith("q"):
        monkeypatch.setenv("BB_LANE_QUICK", budget[1:])
    else:
        monkeypatch.setenv("BB_LANE_BUDGET", budget)
    terms = _run_parity(n=64, steps=120, seed=4242, p_invalid=0.05, act_seed=9)
    assert terms > 20


@pytest.mark.parametrize("kernels", ["1", "2"])
def test_vec_env_all_invalid_and_edge_actions(cuda, kernels, monkeypatch):
    monkeypatch.setenv("BB_STEP_KERNELS", kernels)  # 1: fused (rollout kernel, T = 1); 2: step + escalate
    _run_parity(n=16, steps=20, seed=123, p_invalid=1.0, act_seed=5)


@pytest.mark.parametrize("kernels", ["1", "2"])
def test_vec_env_reset_with_new_seed(cuda, kernels, monkeypatch):
    monkeypatch.setenv("BB_STEP_KERNELS", kernels)  # 1: fused (rollout kernel, T = 1); 2: step + escalate
    from environment.wrappers import VectorizedBlockBlastEnv

    gpu = VectorizedBlockBlastEnv(8, seed=1, device="cuda:0")
    cpu = O.VecEnv(8, seed=1)
    rng = np.random.default_rng(0)
    oc, _ = cpu.reset()
    gpu.reset()
    for _ in range(10):
        a = _actions(rng, oc["action_mask"], 0.0)
        gpu.step(a)
        oc, *_ = cpu.step(a)
    og, _ = gpu.reset(seed=1000)
    oc, _ = cpu.reset(seed=1000)
    for k in og:
        assert np.array_equal(og[k], oc[k])
    for _ in range(40):  # later auto-resets re-seed with 1000 + i
        a = _actions(rng, oc["action_mask"], 0.0)
        og, rg, tg, _, _ = gpu.step(a)
        oc, rc, tc, _, _ = cpu.step(a)
        assert np.array_equal(og["board"], oc["board"]) and np.array_equal(rg, rc) and np.array_equal(tg, tc)
    gpu.close()


@pytest.mark.parametrize("kernels", ["1", "2"])
def test_fused_random_policy_matches_oracle(cuda, kernels, monkeypatch):
    monkeypatch.setenv("BB_STEP_KERNELS", kernels)  # 1: fused (rollout kernel, T = 1); 2: step + escalate
    """bb_step's fused next_action == oracle Philox policy on the post-step mask."""
    from runtime.device_env import DeviceEnvBatch

    n = 512
    dev = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device="cuda:0", env_offset=1000)
    dev.reset()
    mbits = torch.zeros((n, 3), dtype=torch.int64, device=cuda)
    mask = torch.zeros((n, 192), dtype=torch.int8, device=cuda)
    act = torch.zeros(n, dtype=torch.int32, device=cuda)
    nxt = torch.zeros(n, dtype=torch.int32, device=cuda)
    dev.obs(mask_bits=mbits, mask_i8=mask)
    dev.random_actions(mbits, act, seed=0xB10C, step=0)
    exp = philox.random_policy(mask.cpu().numpy().astype(bool), 0xB10C, 0, env_offset=1000)
    assert np.array_equal(act.cpu().numpy(), exp)
    for t in range(1, 30):
        dev.step(act, next_action=nxt, policy_seed=0xB10C, policy_step=t)
        dev.obs(mask_i8=mask)
        exp = philox.random_policy(mask.cpu().numpy().astype(bool), 0xB10C, t, env_offset=1000)
        assert np.array_equal(nxt.cpu().numpy(), exp), t
        assert (dev.reward.cpu().numpy() != -10.0).all()  # policy only picks legal moves
        act, nxt = nxt, act
    dev.close()


@pytest.mark.parametrize("kernels", ["1", "2"])
def test_hard_boards_escalate_to_wave_solver(cuda, kernels, monkeypatch):
    monkeypatch.setenv("BB_STEP_KERNELS", kernels)  # 1: fused (rollout kernel, T = 1); 2: step + escalate
    """Crowded boards make many hand draws exceed the per-lane budget; the
    wave-cooperative path must give the same piece stream as the oracle."""
    from environment.wrappers import VectorizedBlockBlastEnv

    n = 128
    gpu = VectorizedBlockBlastEnv(n, seed=9000, device="cuda:0")
    cpu = O.VecEnv(n, seed=9000)
    gpu.reset()
    oc, _ = cpu.reset()
    rng = np.random.default_rng(11)
    # a policy that piles pieces into the top-left keeps boards crowded
    for t in range(150):
        masks = oc["action_mask"].astype(bool)
        acts = np.array([np.nonzero(m)[0][0] if m.any() else 0 for m in masks])
        flip = rng.random(n) < 0.3
        acts[flip] = [rng.choice(np.nonzero(m)[0]) if m.any() else 0 for m in masks[flip]]
        og, rg, tg, _, _ = gpu.step(acts)
        oc, rc, tc, _, _ = cpu.step(acts)
        assert np.array_equal(og["pieces"], oc["pieces"]), t
        assert np.array_equal(rg.view(np.uint32), rc.view(np.uint32)), t
        assert np.array_equal(tg, tc), t
    gpu.close()
