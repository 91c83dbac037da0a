"""Pin the C oracle (oracle/bb_oracle.c) before the GPU parity tests trust it
at BASELINE's full sizes.

* numpy stream: SeedSequence -> PCG64 words and integers(0, n) draws against
  numpy itself (numpy is a dependency of the reference, not the reference);
* the seed-42 golden of the reference (SURVEY.md section 8(c),
  tests/golden/golden_seed42.json): first hand and play_random_game(42);
* the pure-Python cell-loop oracle (oracle/bb_game.py, pinned by
  test_oracle_golden.py): bit-identical rewards, terminations, masks and
  states under the synthetic policy, with invalid actions, custom rewards and
  without auto-reset;
* the hand-generation DFS verdict against the Python restatement on random
  boards (engine.py:174-224).
"""
import json
import os

import numpy as np
import pytest

from oracle import bb_game as O
from oracle import c_oracle as CO
from oracle import philox

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden_seed42.json")
SEED = 0xB10C


@pytest.mark.parametrize("seed", [0, 1, 42, 2 ** 32 - 1, 2 ** 32, 2 ** 40 + 7, 2 ** 63 + 5, 2 ** 64 - 1])
def test_pcg64_seeding_matches_numpy(seed):
    st = np.random.PCG64(seed).state["state"]
    w = CO.pcg64_seed(seed)
    assert (w[0] << 64 | w[1]) == st["state"] and (w[2] << 64 | w[3]) == st["inc"]


@pytest.mark.parametrize("seed,bound", [(0, 37), (42, 37), (7, 192), (12345, 5), (99, 1), (3, 2 ** 31 + 11)])
def test_bounded_draws_match_numpy(seed, bound):
    ref = np.random.default_rng(seed).integers(0, bound, size=2000)
    assert np.array_equal(CO.rng_draws(seed, bound, 2000).astype(np.int64), ref)


def test_seed42_golden():
    with open(GOLDEN) as f:
        g = json.load(f)
    st, first = CO.play_random_game(42)
    assert first == g["initial_hand_ids"]
    for k, v in g["play_random_game_42"].items():
        assert st[k] == v, k


def test_random_games_match_python_oracle():
    for s in range(6):
        st, _ = CO.play_random_game(s)
        assert st == O.play_random_game(s), s


def _compare_state(py, c):
    ps, cs = py.packed_state(), c.state()
    assert np.array_equal(ps["board"], cs["board"])
    hand = cs["hand"]
    for k in range(3):
        assert np.array_equal(ps["hand"][:, k], (hand >> np.uint32(6 * k)) & np.uint32(63))
        assert np.array_equal(ps["used"][:, k], ((hand >> np.uint32(18 + k)) & np.uint32(1)).astype(bool))
    assert np.array_equal(ps["over"], ((hand >> np.uint32(21)) & np.uint32(1)).astype(bool))
    for k in ("score", "moves", "lines", "combo", "max_combo", "blocks"):
        assert np.array_equal(ps[k].astype(np.int64), cs[k].astype(np.int64)), k
    for i, e in enumerate(py.envs):
        assert cs["prev_holes"][i] == e.prev_holes
        assert 1.0 - cs["prev_center"][i] / 16.0 == e.prev_center


@pytest.mark.parametrize("offset", [0, 1000])
def test_rollout_matches_python_oracle(offset):
    n, T = 48, 70
    py = O.VecEnv(n, seed=42 + offset)
    oc, _ = py.reset()
    c = CO.CVecEnv(np.arange(42 + offset, 42 + offset + n))
    c.reset()
    assert np.array_equal(c.state()["mask"], _bits(oc["action_mask"]))
    acts = philox.random_policy(oc["action_mask"].astype(bool), SEED, 0, env_offset=offset)
    out = c.rollout(T, acts, env_offset=offset)
    for t in range(T):
        assert np.array_equal(out["actions"][t], acts)
        oc, r, term, _, _ = py.step(acts)
        assert np.array_equal(out["reward"][t].view(np.uint32), r.view(np.uint32)), t
        assert np.array_equal(out["terminated"][t].astype(bool), term), t
        assert np.array_equal(out["mask"][t], _bits(oc["action_mask"])), t
        acts = philox.random_policy(oc["action_mask"].astype(bool), SEED, t + 1, env_offset=offset)
    assert np.array_equal(out["next_action"], acts)
    _compare_state(py, c)


def _bits(mask_i8):
    m = np.asarray(mask_i8).astype(bool).reshape(-1, 3, 64)
    w = (1 << np.arange(64, dtype=np.uint64)).astype(np.uint64)
    return (m.astype(np.uint64) * w).sum(axis=2, dtype=np.uint64)


def test_step_invalid_actions_custom_rewards_no_autoreset():
    n, T = 32, 50
    rw = {"line_clear_base": 2.5, "block_placed": 0.03, "game_over_penalty": -3.0, "hole_penalty": -0.25,
          "center_bonus": 0.7, "combo_multiplier_bonus": 1.25, "survival_bonus": 0.0625}
    for autoreset in (True, False):
        py = O.VecEnv(n, seed=7, reward_config=rw)
        oc, _ = py.reset()
        c = CO.CVecEnv(np.arange(7, 7 + n), reward_config=rw, autoreset=autoreset)
        c.reset()
        rng = np.random.default_rng(3)
        for t in range(T):
            masks = oc["action_mask"].astype(bool)
            acts = np.array([rng.choice(np.nonzero(m)[0]) if m.any() else 0 for m in masks], np.int32)
            bad = rng.random(n) < 0.2
            acts[bad] = rng.integers(-3, 195, size=int(bad.sum()))
            o = c.step(acts)
            if autoreset:
                oc, r, term, _, _ = py.step(acts)
            else:  # the single-env semantics: no reset on termination
                rs, ts = [], []
                for e, a in zip(py.envs, acts):
                    _, r1, t1, _, _ = e.step(int(a))
                    rs.append(r1)
                    ts.append(t1)
                r = np.array(rs, np.float64)
                term = np.array(ts)
                oc = {"action_mask": np.stack([e.obs()["action_mask"] for e in py.envs])}
            if autoreset:  # the vec env stores f32 (wrappers.py:88,105)
                assert np.array_equal(o["reward"].view(np.uint32), np.asarray(r, np.float32).view(np.uint32)), t
            else:  # BlockBlastEnv returns the fp64 value
                assert np.array_equal(o["reward_f64"], r), t
            assert np.array_equal(o["terminated"].astype(bool), term), t
            assert np.array_equal(o["mask"], _bits(oc["action_mask"])), t
        _compare_state(py, c)


def test_dfs_verdict_matches_python_restatement():
    rng = np.random.default_rng(11)
    boards, hands = [], []
    for _ in range(600):
        fill = rng.uniform(0.3, 0.8)
        boards.append(int(sum(1 << k for k in range(64) if rng.random() < fill)))
        hands.append(int(rng.integers(0, 37)) | int(rng.integers(0, 37)) << 6 | int(rng.integers(0, 37)) << 12)
    got = CO.solvable_many(np.array(boards, np.uint64), np.array(hands, np.uint32))
    eng = O.Engine(seed=0)
    exp = []
    for b, h in zip(boards, hands):
        eng.hand = [h & 63, (h >> 6) & 63, (h >> 12) & 63]
        exp.append(eng._solvable(O.u64_to_grid(b), [False, False, False]))
    assert np.array_equal(got, np.array(exp))
    assert 0 < got.sum() < len(got)  # both verdicts occur


def test_thread_count_does_not_change_results():
    n, T = 512, 40
    outs = []
    for th in (1, 4):
        c = CO.CVecEnv(np.arange(42, 42 + n))
        c.reset(threads=th)
        a = c.random_actions(c.state()["mask"], SEED, 0)
        outs.append((c.rollout(T, a, threads=th), c.state()))
    for k in ("reward", "terminated", "lines", "actions", "mask"):
        assert np.array_equal(outs[0][0][k], outs[1][0][k]), k
    for k in outs[0][1]:
        assert np.array_equal(outs[0][1][k], outs[1][1][k]), k
