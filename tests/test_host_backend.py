"""The host backend of the env C-ABI (libbbvec_host.so, csrc/bb_host.cpp; SURVEY
§2.2 N10) against the C oracle, bit for bit, on the CPU (no GPU involved).

The backend is selected only by asking for it (device="cpu"); these tests are
the place it runs.  Covered: the fused-policy rollout (bb_rollout) over
several launches with auto-reset re-seeding and unseeded envs; bb_step with
illegal actions, a custom reward config and no auto-reset (single-env
semantics); the final score / moves outputs; observations; the info record;
get/set state; the Gym-surface classes on the backend vs the Python oracle.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import bb_game as O
from oracle import c_oracle as CO

SEED = 0xB10C


@pytest.fixture(scope="module")
def host():
    from runtime import lib as L
    from runtime.build import build_host_lib

    build_host_lib(verbose=False)
    return L.load_host()


def _env(n, offset=0, unseeded=None, reward_config=None, autoreset=True):
    from runtime.device_env import DeviceEnvBatch

    seeds = np.arange(42 + offset, 42 + offset + n, dtype=np.uint64)
    env = DeviceEnvBatch(n, seeds=[int(s) for s in seeds], device="cpu", env_offset=offset,
                         reward_config=reward_config, autoreset=autoreset)
    if unseeded is not None:  # raw PCG words = default_rng(seed) words, seed_value None
        has = np.where(unseeded, 0, 1).astype(np.uint8)
        raw = np.array([CO.pcg64_seed(int(s)) for s in seeds], dtype=np.uint64)
        assert env.lib.bb_seed(env.handle, seeds.ctypes.data_as(C.c_void_p), has.ctypes.data_as(C.c_void_p),
                               raw.ctypes.data_as(C.c_void_p)) == 0
    env.reset()
    cpu = CO.CVecEnv(seeds, reward_config=reward_config, autoreset=autoreset,
                     has_seed=None if unseeded is None else np.where(unseeded, 0, 1))
    cpu.reset()
    return env, cpu


def _same_state(h, c):
    hs, cs = h.state(), c.state()
    for k in ("board", "hand", "score", "combo", "max_combo", "moves", "lines", "blocks", "prev_holes",
              "prev_center"):
        assert np.array_equal(hs[k], cs[k]), f"state {k}"
    assert np.array_equal(hs["rng"][:, :2], cs["rng"][:, :2]), "pcg state"
    return cs


@pytest.mark.parametrize("offset,unseeded", [(0, False), (3 * 65536, True)])
def test_rollout_matches_c_oracle(host, offset, unseeded):
    n, T = 2048, 128
    mask = (np.arange(n) % 2 == 1) if unseeded else None
    env, cpu = _env(n, offset, unseeded=mask)
    cs = _same_state(env, cpu)
    a = torch.from_numpy(cpu.random_actions(cs["mask"], SEED, 0, env_offset=offset))
    ca = a.numpy().copy()
    nxt = torch.zeros_like(a)
    rew = torch.zeros((T, n))
    term = torch.zeros((T, n), dtype=torch.uint8)
    lines = torch.zeros((T, n), dtype=torch.uint8)
    acts = torch.zeros((T, n), dtype=torch.int32)
    masks = torch.zeros((T, n, 3), dtype=torch.int64)
    ends = 0
    for k in range(2):
        env.rollout(T, a, rew, term, lines=lines, actions_out=acts, mask_out=masks, next_action=nxt,
                    policy_seed=SEED, policy_step0=k * T)
        a, nxt = nxt, a
        ref = cpu.rollout(T, ca, policy_seed=SEED, policy_step0=k * T, env_offset=offset)
        ca = ref["next_action"]
        assert np.array_equal(rew.numpy().view(np.uint32), ref["reward"].view(np.uint32)), k
        assert np.array_equal(term.numpy(), ref["terminated"]), k
        assert np.array_equal(lines.numpy(), ref["lines"]), k
        assert np.array_equal(acts.numpy(), ref["actions"]), k
        assert np.array_equal(masks.numpy().view(np.uint64), ref["mask"]), k
        assert np.array_equal(a.numpy(), ca), k
        ends += int(ref["terminated"].sum())
    assert ends > 100
    _same_state(env, cpu)
    env.close()


def test_step_custom_rewards_invalid_actions_no_autoreset(host):
    n, steps = 1024, 120
    rw = {"line_clear_base": 2.5, "block_placed": 0.03, "game_over_penalty": -3.0, "hole_penalty": -0.25,
          "center_bonus": 0.7, "combo_multiplier_bonus": 1.25, "survival_bonus": 0.0625}
    env, cpu = _env(n, reward_config=rw, autoreset=False)
    mask = _same_state(env, cpu)["mask"]
    rng = np.random.default_rng(5)
    for t in range(steps):
        a = cpu.random_actions(mask, SEED, t)
        bad = rng.random(n) < 0.1
        a[bad] = rng.integers(-2, 200, size=int(bad.sum()))
        env.step(torch.from_numpy(a), want_f64=True, want_lines=True)
        o = cpu.step(a)
        mask = o["mask"]
        assert np.array_equal(env.reward_f64.numpy(), o["reward_f64"]), t
        assert np.array_equal(env.terminated.numpy(), o["terminated"]), t
        assert np.array_equal(env.lines.numpy(), o["lines"]), t
    st = _same_state(env, cpu)
    assert ((st["hand"] >> np.uint32(21)) & np.uint32(1)).any()  # games ended and stayed over
    env.close()


def test_step_outputs_replay_and_observations(host):
    """bb_step with the fused policy, final score / moves and the info record
    against bbo_replay; bb_obs against the oracle's expansion."""
    from runtime.device_env import INFO_DTYPE

    n, T = 512, 96
    env, cpu = _env(n)
    cs = _same_state(env, cpu)
    a = torch.from_numpy(cpu.random_actions(cs["mask"], SEED, 0))
    nxt = torch.zeros(n, dtype=torch.int32)
    mb = torch.zeros((n, 3), dtype=torch.int64)
    fs = torch.full((T, n), -1, dtype=torch.int64)
    fm = torch.full((T, n), -1, dtype=torch.int32)
    snaps, actions, rewards, terms, infos = [], [], [], [], []
    for t in range(T):
        board = torch.zeros(n, dtype=torch.int64)
        hand = torch.zeros(n, dtype=torch.int32)
        env.snapshot(board=board, hand=hand, mask_bits=mb)
        snaps.append((board.numpy().copy(), hand.numpy().copy(), mb.numpy().copy()))
        actions.append(a.numpy().copy())
        env.step(a, want_info=True, next_action=nxt, policy_seed=SEED, policy_step=t + 1, final_score=fs[t],
                 final_moves=fm[t])
        rewards.append(env.reward.numpy().copy())
        terms.append(env.terminated.numpy().copy())
        infos.append(env.info_host().copy())
        a, nxt = nxt.clone(), a
    ref = cpu.replay(np.stack(actions))
    assert np.array_equal(np.stack([s[0] for s in snaps]).view(np.uint64), ref["board"])
    assert np.array_equal(np.stack([s[1] for s in snaps]).view(np.uint32), ref["hand"])
    assert np.array_equal(np.stack([s[2] for s in snaps]).view(np.uint64), ref["mask"])
    assert np.array_equal(np.stack(rewards).view(np.uint32), ref["reward"].view(np.uint32))
    d = np.stack(terms).astype(bool)
    assert np.array_equal(d, ref["terminated"].astype(bool)) and d.sum() > 20
    assert np.array_equal(fs.numpy()[d], ref["ep_score"][d]) and (fs.numpy()[~d] == -1).all()
    assert np.array_equal(fm.numpy()[d], ref["ep_moves"][d]) and (fm.numpy()[~d] == -1).all()
    info = np.stack(infos).view(INFO_DTYPE).reshape(T, n)
    assert np.array_equal(info["score"][d], ref["ep_score"][d])
    assert np.array_equal(((info["flags"] >> 1) & 1).astype(bool), d)
    # observations of the final state: board plane, unused pieces, int8 mask
    from oracle import bb_ppo as OP

    x = torch.zeros((n, 4, 8, 8))
    mi = torch.zeros((n, 192), dtype=torch.int8)
    env.obs(x=x, mask_i8=mi, mask_bits=mb)
    st = env.state()
    b, p, mk = OP.expand_packed(st["board"], st["hand"], mb.numpy().view(np.uint64))
    assert np.array_equal(x.numpy()[:, 0], b) and np.array_equal(x.numpy()[:, 1:], p)
    assert np.array_equal(mi.numpy(), mk.astype(np.int8))
    env.close()


def test_set_state_roundtrip(host):
    env, _ = _env(64)
    st = env.state()
    rng = np.random.default_rng(0)
    board = rng.integers(0, 2 ** 63, 64, dtype=np.int64).astype(np.uint64) & np.uint64(0x00FF00FF00FF00FF)
    env.set_state(board=board, score=np.arange(64, dtype=np.int64))
    st2 = env.state()
    assert np.array_equal(st2["board"], board) and np.array_equal(st2["score"], np.arange(64))
    assert np.array_equal(st2["hand"], st["hand"])
    mb = torch.zeros((64, 3), dtype=torch.int64)
    env.obs(mask_bits=mb)
    ref = CO.CVecEnv(np.arange(42, 106, dtype=np.uint64))
    ref.reset()
    ref.set_board_hand(board=board)
    assert np.array_equal(mb.numpy().view(np.uint64), ref.state()["mask"])  # the mask follows the new board
    env.close()


def test_gym_surface_on_host_backend_matches_python_oracle(host):
    from environment.wrappers import VectorizedBlockBlastEnv

    n = 16
    h = VectorizedBlockBlastEnv(n, seed=42, device="cpu")
    o = O.VecEnv(n, seed=42)
    oh, _ = h.reset()
    oo, _ = o.reset()
    rng = np.random.default_rng(7)
    for t in range(60):
        for k in ("board", "pieces", "action_mask"):
            assert np.array_equal(oh[k], oo[k]), (k, t)
        acts = np.array([rng.choice(np.nonzero(m)[0]) for m in oo["action_mask"].astype(bool)])
        oh, rh, th, _, ih = h.step(acts)
        oo, ro, to, _, io = o.step(acts)
        assert np.array_equal(rh.view(np.uint32), ro.view(np.uint32)) and np.array_equal(th, to), t
        for i in range(n):
            assert ih[i]["score"] == io[i]["score"] and ih[i]["moves"] == io[i]["moves"]
    h.close()


def test_host_library_exports_the_env_abi(host):
    from runtime import lib as L

    assert host.bb_abi_version() == L.ABI_VERSION
    for name in L.HOST_SYMBOLS:
        assert hasattr(host, name)
    # the GPU library stays the default: a CPU request never reaches it, a missing GPU is an error
    from runtime.device_env import resolve_device

    assert resolve_device("cpu").type == "cpu"
    if not torch.cuda.is_available():
        with pytest.raises(L.BBNativeError):
            resolve_device(None)
