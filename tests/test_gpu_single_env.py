"""GPU parity of the single-env Gym surface (BlockBlastEnv, N = 1, no
auto-reset) against the oracle, plus the reference's tests/test_environment.py
checks restated."""
import numpy as np
import pytest

from oracle import bb_game as O

pytestmark = pytest.mark.gpu


def test_full_game_fp64_reward_exact(cuda):
    from environment.block_blast_env import BlockBlastEnv

    for seed in (42, 5, 77):
        env = BlockBlastEnv(seed=seed)
        ref = O.Env(seed=seed)
        og, ig = env.reset()
        oc, ic = ref.reset()
        assert ig == ic
        rng = np.random.default_rng(seed)
        done = False
        steps = 0
        while steps < 400:
            m = oc["action_mask"]
            if rng.random() < 0.15:
                a = int(rng.integers(-3, 200))
            else:
                valid = np.nonzero(m)[0]
                a = int(rng.choice(valid)) if valid.size else 0
            og, rg, tg, trg, ig = env.step(a)
            oc, rc, tc, trc, ic = ref.step(a)
            assert type(rg) is float and rg == rc, (steps, rg, rc)  # fp64 bit-exact
            assert type(tg) is bool and tg == tc and trg is False
            assert ig == ic, (steps, ig, ic)
            for k in og:
                assert np.array_equal(og[k], oc[k]), k
            steps += 1
            if tc:
                done = True
                break
        assert done
        # after game over every action is invalid (engine.py:342)
        _, r, t, _, info = env.step(int(np.nonzero(oc["action_mask"] == 0)[0][0]))
        assert r == -10.0 and info["invalid_action"] and t is False


def test_reference_environment_checks(cuda):
    from environment.block_blast_env import BlockBlastEnv, BlockBlastEnvFlat
    from environment.wrappers import VectorizedBlockBlastEnv

    env = BlockBlastEnv()
    assert (env.BOARD_SIZE, env.NUM_PIECES_PER_TURN, env.ACTION_SPACE_SIZE) == (8, 3, 192)
    assert env.action_space.n == 192
    assert {"board", "pieces", "action_mask"} <= set(env.observation_space.spaces)
    obs, info = env.reset()
    assert obs["board"].shape == (8, 8) and obs["pieces"].shape == (3, 8, 8) and obs["action_mask"].shape == (192,)
    e1, e2 = BlockBlastEnv(seed=42), BlockBlastEnv(seed=42)
    assert np.array_equal(e1.reset()[0]["pieces"], e2.reset()[0]["pieces"])
    o1, _ = env.reset(seed=42)
    o2, _ = env.reset(seed=42)
    assert np.array_equal(o1["pieces"], o2["pieces"])
    mask = env.get_action_mask()
    assert mask.shape == (192,) and mask.dtype == bool and mask.sum() > 0
    a = env.sample_valid_action()
    assert mask[a]
    assert all(0 <= x < 192 for x in env.get_valid_actions())
    _, r, t, tr, info = env.step(a)
    assert isinstance(r, float) and isinstance(t, bool) and isinstance(tr, bool) and r > -100
    assert "score" in info and "moves" in info
    assert env._action_to_move(128) == (2, 0, 0) and env._move_to_action(0, 7, 7) == 63
    out = BlockBlastEnv(render_mode="ansi")
    out.reset()
    assert isinstance(out.render(), str) and len(out.render()) > 0
    flat = BlockBlastEnvFlat()
    fo, _ = flat.reset()
    assert "obs" in flat.observation_space.spaces and fo["obs"].shape == (178,)
    v = VectorizedBlockBlastEnv(num_envs=4)
    vo, vi = v.reset()
    assert vo["board"].shape == (4, 8, 8) and vo["pieces"].shape == (4, 3, 8, 8) and len(vi) == 4
    acts = v.sample_valid_actions()
    assert len(acts) == 4
    vo, vr, vt, vtr, vi = v.step(acts)
    assert len(vr) == 4 and len(vt) == 4 and v.get_action_masks().shape == (4, 192)
    v.close()


def test_episode_terminates(cuda):
    from environment.block_blast_env import BlockBlastEnv

    env = BlockBlastEnv()
    env.reset(seed=42)
    for _ in range(1000):
        _, _, t, tr, _ = env.step(env.sample_valid_action())
        if t or tr:
            break
    assert t
