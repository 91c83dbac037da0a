"""CPU checks of the oracle's PPO-update restatement (oracle/bb_ppo.py) used
by tests/test_gpu_ppo_update_oracle.py: a small network through ppo_update
with its per-step hooks, the packed-observation expansion against the Python
oracle's own get_observation, and the float64 clipped gradients."""
import copy

import numpy as np
import torch

from oracle import bb_game as G
from oracle import bb_ppo as OP


class _Cfg:
    gamma, gae_lambda, clip_epsilon, value_coef, entropy_coef, max_grad_norm = 0.99, 0.95, 0.2, 0.5, 0.01, 0.5
    learning_rate, num_epochs, batch_size = 3e-4, 2, 16


def _buffer(T=4, N=8, seed=0):
    rng = np.random.default_rng(seed)
    env = G.VecEnv(N, seed=42)
    obs, _ = env.reset()
    buf = {k: [] for k in ("boards", "pieces", "action_masks", "actions", "log_probs", "rewards", "dones", "values")}
    for _ in range(T):
        m = obs["action_mask"].astype(bool)
        a = np.array([rng.choice(np.nonzero(x)[0]) for x in m])
        buf["boards"].append(obs["board"].astype(np.float32))
        buf["pieces"].append(obs["pieces"].astype(np.float32))
        buf["action_masks"].append(obs["action_mask"].astype(np.float32))
        buf["actions"].append(a.astype(np.int64))
        buf["log_probs"].append(-rng.random(N).astype(np.float32) * 3)
        buf["values"].append(rng.standard_normal(N).astype(np.float32))
        obs, r, term, _, _ = env.step(a)
        buf["rewards"].append(r.astype(np.float32))
        buf["dones"].append(term.astype(np.float32))
    return {k: np.stack(v) for k, v in buf.items()}


def test_ppo_update_hooks_and_fp64_grads():
    torch.manual_seed(0)
    net = OP.ReferenceNetwork(conv_channels=(8, 16, 16), fc_hidden=(32, 16), dropout=0.0)
    buf = _buffer()
    cfg = _Cfg()
    seen = []
    opt = torch.optim.Adam(net.parameters(), lr=cfg.learning_rate, eps=1e-5)
    rng = np.random.default_rng(3)
    means, per, adv, ret = OP.ppo_update(net, opt, buf, np.zeros(8, np.float32), cfg, rng.permutation,
                                         before_step=lambda k: seen.append(("b", k)),
                                         after_step=lambda k, row, batch: seen.append(("a", k, len(batch))))
    assert per.shape == (4, 6) and np.isfinite(per).all()
    assert seen == [x for k in range(4) for x in (("b", k), ("a", k, 7))]
    assert abs(means["total_loss"] - per[:, 3].mean()) < 1e-12
    np.testing.assert_array_equal(ret, adv + buf["values"])
    # float64 gradients agree with float32 ones to fp32 rounding
    batch = next(OP.get_samples(dict(buf, advantages=adv, returns=ret), 16, np.arange(32)))
    g32 = OP.clipped_grads(net, batch, cfg)
    g64 = OP.clipped_grads(copy.deepcopy(net).double(), batch, cfg)
    total = float(torch.sqrt(sum((g ** 2).sum() for g in g64.values())))
    for k, v in g32.items():  # (a conv bias feeding a BatchNorm has a true gradient of 0: absolute bound)
        assert float((v.double() - g64[k]).norm()) <= 1e-4 * float(g64[k].norm()) + 1e-6 * total, k


def test_expand_packed_matches_python_oracle_observation():
    env = G.VecEnv(16, seed=42)
    obs, _ = env.reset()
    rng = np.random.default_rng(1)
    for _ in range(5):
        m = obs["action_mask"].astype(bool)
        obs, *_ = env.step(np.array([rng.choice(np.nonzero(x)[0]) for x in m]))
    boards = np.array([G.grid_to_u64(e.engine.grid) for e in env.envs], dtype=np.uint64)
    hands = np.array([sum(p << (6 * s) for s, p in enumerate(e.engine.hand)) |
                      sum(int(u) << (18 + s) for s, u in enumerate(e.engine.used)) for e in env.envs], np.uint32)
    mask = obs["action_mask"].reshape(16, 3, 64).astype(np.uint64)
    bits = (mask << np.arange(64, dtype=np.uint64)).sum(axis=2, dtype=np.uint64)
    b, p, mk = OP.expand_packed(boards, hands, bits)
    np.testing.assert_array_equal(b, obs["board"])
    np.testing.assert_array_equal(p, obs["pieces"])
    np.testing.assert_array_equal(mk, obs["action_mask"].astype(np.float32))
