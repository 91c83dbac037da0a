"""SURVEY 8(f) ranks 3-4 against the oracle, on the GPU (the eval/play path, the flat observation and the
reference wrappers on the real N=1 env).

* Eval (scripts/evaluate.py:23-90): the games ``evaluate_agent`` plays -- batched (one device env per
  episode) and sequential (the reference's loop on ``BlockBlastEnv``) -- are replayed action by action
  through ``oracle.bb_game.Env`` seeded ``seed + episode``.  Every action must be legal in the oracle's
  game, the oracle's game must end exactly at the recorded length, and the score, length, lines cleared
  and max combo that ``evaluate_agent`` reports must equal the oracle's, episode by episode.  The policy
  side is checked too: with ``deterministic=True`` each action must be the argmax of the reference
  network (``oracle.bb_ppo.ReferenceNetwork``, same weights, eval mode, float64) on the oracle's
  observation, or within north_star's 1e-5 fp32 tolerance of it (a near-tie: logit gap
  <= 2e-5 * max(1, |x|)).
* ``BlockBlastEnvFlat`` (block_blast_env.py:326-389): the 178-d observation equals ``Env.flat_obs`` of
  the oracle element for element on every step of several games, game over and invalid actions included.
* ``NormalizedRewardWrapper`` / ``FrameStackWrapper`` / ``make_env`` (wrappers.py:144-309) on the real
  device env against the oracle env + ``oracle.bb_game.ReturnNormalizer`` (an independent fp64 variance
  of the discounted returns, math.fsum from scratch) + ``FrameStack``: stacked boards, pieces and mask
  bit-equal, ``raw_reward`` bit-equal to the oracle's fp64 reward, the normalised reward within 1e-12
  relative, terminations equal, over several episodes (the statistics persist across resets).
"""
import copy

import numpy as np
import pytest
import torch

from oracle import bb_game as O
from oracle import bb_ppo as OP

pytestmark = pytest.mark.gpu


def _replay(actions, seed):
    """The oracle's game for one recorded episode: (score, length, lines, max_combo, observations)."""
    env = O.Env(seed=seed)
    obs, _ = env.reset(seed=seed)
    seen = [obs]
    term = False
    for t, a in enumerate(actions):
        assert not term, ("the oracle's game ended before the recorded episode", t)
        assert obs["action_mask"][a] == 1, ("illegal action in the oracle's game", t, a)
        obs, _, term, _, info = env.step(a)
        seen.append(obs)
    assert term, "the recorded episode ended but the oracle's game did not"
    return info["score"], len(actions), info["lines_cleared"], info["max_combo"], seen[:-1]


def _check_argmax(agent, obs_list, actions):
    """Each deterministic action is the fp64 reference network's argmax up to a 1e-5 near-tie."""
    ref = OP.ReferenceNetwork(dropout=0.0)
    ref.load_state_dict({k: v.detach().cpu() for k, v in agent.network.state_dict().items()})
    net = copy.deepcopy(ref).double().eval()
    b = torch.from_numpy(np.stack([o["board"] for o in obs_list])).double()
    p = torch.from_numpy(np.stack([o["pieces"] for o in obs_list])).double()
    m = torch.from_numpy(np.stack([o["action_mask"] for o in obs_list])).double()
    with torch.no_grad():
        lg, _ = net(b, p, m)
    lg = lg.numpy()
    a = np.asarray(actions)
    best = lg.max(1)
    gap = best - lg[np.arange(len(a)), a]
    scale = np.maximum(1.0, np.abs(best))
    ties = int((gap > 0).sum())
    assert (gap <= 2e-5 * scale).all(), (np.nonzero(gap > 2e-5 * scale)[0], gap.max())
    return ties


@pytest.mark.parametrize("batched", [True, False])
def test_eval_episodes_replay_through_oracle(cuda, batched):
    from agents import PPOAgent, PPOConfig
    from evaluation.evaluate import _evaluate_sequential, evaluate_agent

    torch.manual_seed(5)
    agent = PPOAgent(PPOConfig(), device=cuda, sample_seed=0)
    seed, n = 17, 8 if batched else 4
    if batched:
        res = evaluate_agent(agent, num_episodes=n, deterministic=True, seed=seed, record_actions=True)
    else:
        agent.eval()
        res = _evaluate_sequential(agent, n, True, False, seed, record_actions=True)
    obs_all, act_all, lines, combos = [], [], [], []
    for ep in range(n):
        score, length, ln, combo, seen = _replay(res["actions"][ep], seed + ep)
        assert res["scores"][ep] == score, (ep, res["scores"][ep], score)
        assert res["lengths"][ep] == length, ep
        obs_all += seen
        act_all += res["actions"][ep]
        lines.append(ln)
        combos.append(combo)
    assert res["mean_lines_cleared"] == np.mean(lines) and res["mean_max_combo"] == np.mean(combos)
    assert res["mean_score"] == np.mean(res["scores"]) and res["max_score"] == max(res["scores"])
    assert res["num_episodes"] == n and min(res["lengths"]) > 0
    ties = _check_argmax(agent, obs_all, act_all)
    print(f"{'batched' if batched else 'sequential'} eval: {n} episodes, {len(act_all)} moves replayed "
          f"through the oracle; {ties} argmax near-ties within 1e-5")


def test_eval_stochastic_episodes_replay_through_oracle(cuda):
    """Sampled (deterministic=False) evaluation: the env side of every game equals the oracle's."""
    from agents import PPOAgent, PPOConfig
    from evaluation.evaluate import evaluate_agent

    torch.manual_seed(6)
    agent = PPOAgent(PPOConfig(), device=cuda, sample_seed=3)
    res = evaluate_agent(agent, num_episodes=16, deterministic=False, seed=100, record_actions=True)
    for ep in range(16):
        score, length, lines, combo, _ = _replay(res["actions"][ep], 100 + ep)
        assert (res["scores"][ep], res["lengths"][ep]) == (score, length), ep


def test_flat_observation_matches_oracle(cuda):
    from environment.block_blast_env import BlockBlastEnvFlat

    rng = np.random.default_rng(9)
    for seed in (42, 7, 1234):
        env = BlockBlastEnvFlat(seed=seed, device=cuda)
        ora = O.Env(seed=seed)
        obs, _ = env.reset()
        ora.reset()
        assert obs["obs"].shape == (178,) and obs["obs"].dtype == np.float32
        for t in range(400):
            want = ora.flat_obs()
            np.testing.assert_array_equal(obs["obs"], want["obs"], err_msg=f"seed {seed} step {t}")
            np.testing.assert_array_equal(obs["action_mask"], want["action_mask"])
            legal = np.nonzero(want["action_mask"])[0]
            if legal.size == 0 or t % 37 == 5:
                a = int(rng.integers(0, 192))  # invalid actions (and every action after game over)
            else:
                a = int(rng.choice(legal))
            obs, r, term, _, info = env.step(a)
            _, r_o, term_o, _, info_o = ora.step(a)
            assert (r, term) == (r_o, term_o) and info["invalid_action"] == info_o["invalid_action"], (seed, t)
            if term:
                np.testing.assert_array_equal(obs["obs"], ora.flat_obs()["obs"])
                a = int(rng.integers(0, 192))  # after game over every action is invalid on both sides
                obs, r, term2, _, info = env.step(a)
                _, r_o, term_o, _, info_o = ora.step(a)
                assert (r, term2, info["invalid_action"]) == (r_o, term_o, info_o["invalid_action"]) == (
                    -10.0, False, True)
                np.testing.assert_array_equal(obs["obs"], ora.flat_obs()["obs"])
                obs, _ = env.reset()
                ora.reset()
        env.close()


def test_reference_wrappers_on_real_env_match_oracle(cuda):
    from environment import FrameStackWrapper, NormalizedRewardWrapper, make_env

    seed, frames = 3, 4
    env = make_env(seed=seed, normalize_reward=True, frame_stack=frames)
    assert isinstance(env, NormalizedRewardWrapper) and isinstance(env.env, FrameStackWrapper)
    ora, norm, stack = O.Env(seed=seed), O.ReturnNormalizer(), O.FrameStack(frames)
    obs, _ = env.reset()
    o, _ = ora.reset()
    norm.reset()
    want_board = stack.reset(o["board"])
    rng = np.random.default_rng(0)
    episodes, steps = 0, 0
    while episodes < 4:
        np.testing.assert_array_equal(obs["board"], want_board)
        np.testing.assert_array_equal(obs["pieces"], o["pieces"])
        np.testing.assert_array_equal(obs["action_mask"], o["action_mask"])
        a = int(rng.choice(np.nonzero(o["action_mask"])[0]))
        obs, r, term, trunc, info = env.step(a)
        o, r_o, term_o, _, _ = ora.step(a)
        want_board = stack.step(o["board"])
        want_r = norm.step(r_o, term_o)
        assert info["raw_reward"] == r_o and term == term_o, steps  # fp64 reward bit for bit
        assert abs(r - want_r) <= 1e-12 * max(1.0, abs(want_r)), (steps, r, want_r)
        steps += 1
        if term:
            episodes += 1
            obs, _ = env.reset()
            o, _ = ora.reset()
            norm.reset()
            want_board = stack.reset(o["board"])
    print(f"wrappers: {episodes} episodes, {steps} steps equal to the oracle")
    env.close()
