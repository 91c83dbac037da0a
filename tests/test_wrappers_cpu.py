"""Reference wrappers (wrappers.py:144-309) on a scripted stand-in env: the
wrapper arithmetic is host-side and needs no GPU."""
import numpy as np

from environment.extra_wrappers import FrameStackWrapper, NormalizedRewardWrapper, RunningMeanStd
from environment.spaces import Box, Dict as DictSpace, Discrete


class _Scripted:
    def __init__(self, rewards):
        self.rewards = list(rewards)
        self.t = 0
        self.observation_space = DictSpace({"board": Box(0.0, 1.0, (8, 8), np.float32),
                                            "pieces": Box(0.0, 1.0, (3, 8, 8), np.float32),
                                            "action_mask": Box(0, 1, (192,), np.int8)})
        self.action_space = Discrete(192)

    def _obs(self):
        return {"board": np.full((8, 8), self.t, np.float32), "pieces": np.zeros((3, 8, 8), np.float32),
                "action_mask": np.ones(192, np.int8)}

    def reset(self, **kw):
        self.t = 0
        return self._obs(), {}

    def step(self, a):
        r = self.rewards[self.t]
        self.t += 1
        return self._obs(), r, self.t == len(self.rewards), False, {}

    def close(self):
        pass


def test_running_mean_std_matches_numpy():
    rng = np.random.default_rng(1)
    xs = [rng.standard_normal(5) * 3 + 1 for _ in range(7)]
    rms = RunningMeanStd()
    for x in xs:
        rms.update(x)
    allx = np.concatenate(xs)
    # the epsilon pseudo-count (1e-4) of the initial (0, 1) moments is all that differs
    assert abs(rms.mean - allx.mean()) < 1e-4 and abs(rms.var - allx.var()) < 1e-3


def test_normalized_reward_wrapper():
    rs = [1.0, 0.5, -1.0, 2.0]
    env = NormalizedRewardWrapper(_Scripted(rs), gamma=0.9)
    env.reset()
    ret, rms = 0.0, RunningMeanStd()
    for i, r in enumerate(rs):
        _, nr, term, _, info = env.step(0)
        ret = ret * 0.9 + r
        rms.update(np.array([ret]))
        assert info["raw_reward"] == r and nr == r / (np.sqrt(rms.var) + 1e-8)
    assert term and env.returns == 0.0


def test_frame_stack_wrapper():
    env = FrameStackWrapper(_Scripted([0.0] * 5), num_frames=3)
    assert env.observation_space["board"].shape == (3, 8, 8)
    obs, _ = env.reset()
    assert obs["board"].shape == (3, 8, 8) and (obs["board"] == 0).all()
    obs, *_ = env.step(0)
    obs, *_ = env.step(0)
    assert [float(obs["board"][k, 0, 0]) for k in range(3)] == [0.0, 1.0, 2.0]


def test_normalized_reward_wrapper_against_independent_variance():
    """The product's incremental (Chan) variance against the oracle's from-scratch fp64 pooled variance
    (oracle.bb_game.ReturnNormalizer) over several episodes of a scripted env: the statistics persist
    across resets, the normalised rewards agree to 1e-12 relative."""
    import sys
    import os

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import bb_game as O

    rng = np.random.default_rng(4)
    env = NormalizedRewardWrapper(_Scripted(list(rng.standard_normal(25) * 3)), gamma=0.99)
    ora = O.ReturnNormalizer(gamma=0.99)
    for ep in range(6):
        env.reset()
        env.env.rewards = list(rng.standard_normal(int(rng.integers(3, 25))) * (ep + 1))
        ora.reset()
        term = False
        while not term:
            _, nr, term, _, info = env.step(0)
            want = ora.step(info["raw_reward"], term)
            assert abs(nr - want) <= 1e-12 * max(1.0, abs(want)), (ep, nr, want)
    assert len(ora.history) > 30
