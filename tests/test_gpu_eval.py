"""Batched evaluation (one device env per episode, lockstep) equals the
reference's sequential loop (scripts/evaluate.py:23-90) for an argmax policy,
and the reference wrappers run on the N=1 env."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_batched_evaluation_equals_sequential(cuda):
    from agents import PPOAgent, PPOConfig
    from evaluation.evaluate import _evaluate_sequential, evaluate_agent

    torch.manual_seed(0)
    agent = PPOAgent(PPOConfig(), device=cuda, sample_seed=0)
    res_b = evaluate_agent(agent, num_episodes=6, deterministic=True, seed=11)
    res_s = _evaluate_sequential(agent, 6, True, False, 11)
    for k in ("scores", "lengths"):
        assert res_b[k] == res_s[k], k
    for k in ("mean_lines_cleared", "mean_max_combo", "median_score"):
        assert res_b[k] == res_s[k], k
    assert res_b["num_episodes"] == 6 and min(res_b["lengths"]) > 0


def test_reference_wrappers_on_device_env(cuda):
    from environment import FrameStackWrapper, NormalizedRewardWrapper, make_env

    env = make_env(seed=3, normalize_reward=True, frame_stack=4)
    assert isinstance(env, NormalizedRewardWrapper) and isinstance(env.env, FrameStackWrapper)
    obs, _ = env.reset()
    assert obs["board"].shape == (4, 8, 8) and obs["pieces"].shape == (3, 8, 8)
    rng = np.random.default_rng(0)
    for _ in range(10):
        a = int(rng.choice(np.nonzero(obs["action_mask"])[0]))
        obs, r, term, trunc, info = env.step(a)
        assert "raw_reward" in info and np.isfinite(r)
        if term:
            break
    assert obs["board"].shape == (4, 8, 8)
    env.close()
