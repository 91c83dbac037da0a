"""CPU restatement of the rollout-side PPO math (TEST INFRASTRUCTURE ONLY).

* ``gae``: RolloutBuffer.compute_returns_and_advantages (ppo.py:141-169),
  the reference loop on numpy float32 arrays (numpy-2 promotion rules).
* ``normalize_advantages``: ppo.py:196.
* ``masked_categorical``: BlockBlastNetwork.forward masking + get_action_and_value
  tail + _masked_entropy (network.py:173-180, 210-262) with torch CPU ops;
  sampling is made deterministic by inverse CDF on a supplied uniform (torch's
  multinomial stream is not reproducible across devices -- parity unpinned
  against the reference's own sample, which no reference test pins either).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F
from torch.distributions import Categorical


def gae(rewards, values, dones, last_values, gamma, gae_lambda):
    """ppo.py:155-169 verbatim semantics on [T, N] float32 arrays."""
    T = rewards.shape[0]
    adv = np.zeros_like(rewards, dtype=np.float32)
    last = 0
    for t in reversed(range(T)):
        nnt = 1.0 - dones[t]
        nv = last_values if t == T - 1 else values[t + 1]
        delta = rewards[t] + gamma * nv * nnt - values[t]
        last = delta + gamma * gae_lambda * nnt * last
        adv[t] = last
    return adv, adv + values


def normalize_advantages(adv):
    """ppo.py:196 on the flattened float32 advantages."""
    a = adv.reshape(-1)
    return (a - a.mean()) / (a.std() + 1e-8)


def masked_categorical(logits: np.ndarray, mask: np.ndarray, uniform=None, action=None, deterministic=False):
    """Returns (action int64, log_prob f32, entropy f32) for (N,192) logits."""
    lg = torch.from_numpy(np.asarray(logits, dtype=np.float32))
    mk = torch.from_numpy(np.asarray(mask)).bool()
    masked = lg + torch.where(mk, torch.zeros_like(lg), torch.full_like(lg, float("-inf")))
    probs = F.softmax(masked, dim=-1)
    dist = Categorical(probs=probs)
    if action is None:
        if deterministic:
            action = torch.argmax(probs, dim=-1)
        else:
            P = dist.probs.double().numpy()
            u = np.asarray(uniform, dtype=np.float64)
            cdf = np.cumsum(P, axis=1)
            target = u * cdf[:, -1]
            out = np.zeros(P.shape[0], dtype=np.int64)
            for i in range(P.shape[0]):
                hit = np.nonzero((cdf[i] > target[i]) & mk[i].numpy())[0]
                out[i] = hit[0] if hit.size else np.nonzero(mk[i].numpy())[0][-1]
            action = torch.from_numpy(out)
    else:
        action = torch.as_tensor(action, dtype=torch.int64)
    logp = dist.log_prob(action)
    m = mk.float()
    mp = probs * m
    norm = mp / mp.sum(dim=-1, keepdim=True).clamp(min=1e-10)
    ent = -(norm * torch.log(norm.clamp(min=1e-10)) * m).sum(dim=-1)
    return action.numpy(), logp.numpy().astype(np.float32), ent.numpy().astype(np.float32)
