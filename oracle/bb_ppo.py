"""CPU restatement of the PPO side of the hot path (TEST INFRASTRUCTURE ONLY).

* ``gae``: RolloutBuffer.compute_returns_and_advantages (ppo.py:141-169),
  the reference loop on numpy float32 arrays (numpy-2 promotion rules).
* ``normalize_advantages``: ppo.py:196.
* ``masked_categorical``: BlockBlastNetwork.forward masking + get_action_and_value
  tail + _masked_entropy (network.py:173-180, 210-262) with torch CPU ops;
  sampling is made deterministic by inverse CDF on a supplied uniform (torch's
  multinomial stream is not reproducible across devices -- parity unpinned
  against the reference's own sample, which no reference test pins either).
* ``ReferenceNetwork``: BlockBlastNetwork / ResidualBlock (network.py:14-182)
  as plain torch modules (Conv2d, BatchNorm2d, ReLU, Linear, Dropout), with the
  reference's module indices so state_dicts interchange with the product.
* ``expand_packed``: engine.get_observation (engine.py:478-507) from packed
  board bits / hand words / mask bits, on the oracle's own piece table.
* ``get_samples`` / ``ppo_update``: RolloutBuffer.get_samples (ppo.py:171-213)
  and PPOAgent.update (ppo.py:330-423) on CPU float32 torch, with the
  permutation of each epoch injected (the reference draws it from numpy's
  global RandomState, ppo.py:199) and every minibatch's six statistics kept.

PPO numerics have no reference fixture: they follow numpy / torch semantics
(the reference's own dependencies) op for op -- parity unpinned against the
reference itself, pinned against its algorithm.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Categorical

from . import bb_game as G


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


def categorical_cdf(logits: np.ndarray, mask: np.ndarray) -> np.ndarray:
    """(N,192) float64 running sums of Categorical(probs=softmax(masked logits)).probs -- the CDF the
    inverse-CDF sample of masked_categorical walks (network.py:173-180, 213-228); cdf[:, -1] is the total."""
    lg = torch.from_numpy(np.asarray(logits, dtype=np.float32))
    mk = torch.from_numpy(np.asarray(mask)).bool()
    masked = lg + torch.where(mk, torch.zeros_like(lg), torch.full_like(lg, float("-inf")))
    return np.cumsum(Categorical(probs=F.softmax(masked, dim=-1)).probs.double().numpy(), axis=1)


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
            u = np.asarray(uniform, dtype=np.float64)
            cdf = categorical_cdf(logits, mask)
            target = u * cdf[:, -1]
            out = np.zeros(cdf.shape[0], dtype=np.int64)
            for i in range(cdf.shape[0]):
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


# --------------------------------------------------------------------------
# network.py:14-182
# --------------------------------------------------------------------------
class ResidualBlock(nn.Module):
    """network.py:14-30."""

    def __init__(self, channels: int):
        super().__init__()
        self.conv1 = nn.Conv2d(channels, channels, kernel_size=3, padding=1)
        self.bn1 = nn.BatchNorm2d(channels)
        self.conv2 = nn.Conv2d(channels, channels, kernel_size=3, padding=1)
        self.bn2 = nn.BatchNorm2d(channels)

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        out = out + x
        return F.relu(out)


class ReferenceNetwork(nn.Module):
    """network.py:43-182 (use_residual, use_batch_norm): conv encoder, FC
    encoder with Dropout(dropout) (the reference's 0.1; tests pass 0 so the
    two sides see the same function), policy and value heads."""

    def __init__(self, conv_channels=(64, 128, 128), fc_hidden=(512, 256), dropout: float = 0.1):
        super().__init__()
        layers, cin = [], 4
        for i, cout in enumerate(conv_channels):
            layers += [nn.Conv2d(cin, cout, kernel_size=3, padding=1), nn.BatchNorm2d(cout), nn.ReLU()]
            if i > 0:
                layers.append(ResidualBlock(cout))
            cin = cout
        self.conv_encoder = nn.Sequential(*layers)
        fc, fin = [], conv_channels[-1] * 64
        for h in fc_hidden:
            fc += [nn.Linear(fin, h), nn.ReLU(), nn.Dropout(dropout)]
            fin = h
        self.fc_encoder = nn.Sequential(*fc)
        self.policy_head = nn.Sequential(nn.Linear(fc_hidden[-1], 256), nn.ReLU(), nn.Linear(256, 192))
        self.value_head = nn.Sequential(nn.Linear(fc_hidden[-1], 128), nn.ReLU(), nn.Linear(128, 1))
        for m in self.modules():  # network.py:122-133
            if isinstance(m, (nn.Linear, nn.Conv2d)):
                nn.init.kaiming_uniform_(m.weight, nonlinearity="relu")
                nn.init.zeros_(m.bias)

    def forward(self, board, pieces, action_mask=None):
        """network.py:135-182."""
        if board.dim() == 3:
            board = board.unsqueeze(1)
        x = torch.cat([board, pieces], dim=1)
        x = self.conv_encoder(x)
        x = x.view(x.size(0), -1)
        x = self.fc_encoder(x)
        logits = self.policy_head(x)
        value = self.value_head(x)
        if action_mask is not None:
            logits = logits + torch.where(action_mask.bool(), torch.zeros_like(logits),
                                          torch.full_like(logits, float("-inf")))
        return logits, value.squeeze(-1)

    def get_action_and_value(self, board, pieces, action_mask, action):
        """network.py:184-230 with a given action (the update's evaluation)."""
        logits, value = self.forward(board, pieces, action_mask)
        probs = F.softmax(logits, dim=-1)
        dist = Categorical(probs)
        log_prob = dist.log_prob(action)
        mask = action_mask.bool()  # _masked_entropy, network.py:232-262
        masked_probs = probs * mask.float()
        prob_sum = masked_probs.sum(dim=-1, keepdim=True).clamp(min=1e-10)
        normalized = masked_probs / prob_sum
        entropy = -(normalized * torch.log(normalized.clamp(min=1e-10)) * mask.float()).sum(dim=-1)
        return action, log_prob, entropy, value


# --------------------------------------------------------------------------
# packed rollout records -> the reference's buffer layout (ppo.py:75-139)
# --------------------------------------------------------------------------
def expand_packed(board_bits, hand, mask_bits):
    """engine.get_observation (engine.py:478-507) of packed states: board u64
    (bit r*8+c), hand word (3 x 6-bit ids, used bits 18-20), mask u64 x 3 ->
    boards f32 [..., 8, 8], pieces f32 [..., 3, 8, 8], masks f32 [..., 192]."""
    b = np.asarray(board_bits).astype(np.uint64)
    h = np.asarray(hand).astype(np.uint32)
    m = np.asarray(mask_bits).astype(np.uint64)
    shape = b.shape
    bit = np.arange(64, dtype=np.uint64)
    boards = ((b.reshape(-1, 1) >> bit) & np.uint64(1)).astype(np.float32).reshape(*shape, 8, 8)
    planes = np.stack([G.piece_mask(p) for p in range(G.NUM_PIECES)])  # pieces.py:39-45
    pieces = np.zeros((int(np.prod(shape)), 3, 8, 8), np.float32)
    hf = h.reshape(-1)
    for s in range(3):
        pid = ((hf >> np.uint32(6 * s)) & np.uint32(63)).astype(np.int64)
        used = ((hf >> np.uint32(18 + s)) & np.uint32(1)).astype(bool)
        pieces[:, s] = np.where(used[:, None, None], np.float32(0), planes[pid])
    masks = ((m.reshape(-1, 3, 1) >> bit) & np.uint64(1)).astype(np.float32).reshape(*shape, 192)
    return boards, pieces.reshape(*shape, 3, 8, 8), masks


# --------------------------------------------------------------------------
# ppo.py:171-213 and 330-423
# --------------------------------------------------------------------------
def get_samples(buf: Dict[str, np.ndarray], batch_size: int, indices: np.ndarray):
    """RolloutBuffer.get_samples (ppo.py:171-213) with the permutation given."""
    T, N = buf["rewards"].shape
    total = T * N
    boards = buf["boards"].reshape(total, *buf["boards"].shape[2:])
    pieces = buf["pieces"].reshape(total, *buf["pieces"].shape[2:])
    masks = buf["action_masks"].reshape(total, -1)
    actions = buf["actions"].reshape(total)
    log_probs = buf["log_probs"].reshape(total)
    advantages = buf["advantages"].reshape(total)
    returns = buf["returns"].reshape(total)
    advantages = (advantages - advantages.mean()) / (advantages.std() + 1e-8)  # ppo.py:196
    for start in range(0, total, batch_size):
        end = min(start + batch_size, total)
        b = indices[start:end]
        yield (torch.from_numpy(boards[b]), torch.from_numpy(pieces[b]), torch.from_numpy(masks[b]),
               torch.from_numpy(actions[b]), torch.from_numpy(log_probs[b]), torch.from_numpy(advantages[b]),
               torch.from_numpy(returns[b]))


STAT_KEYS = ("policy_loss", "value_loss", "entropy", "total_loss", "approx_kl", "clip_fraction")


def minibatch_loss(network: ReferenceNetwork, batch, cfg):
    """ppo.py:364-392: the clipped surrogate, MSE value loss and entropy bonus
    of one minibatch (in the network's dtype)."""
    boards, pieces, masks, actions, old_log_probs, advantages, returns = batch
    dt = next(network.parameters()).dtype
    boards, pieces, masks, old_log_probs, advantages, returns = (
        t.to(dt) for t in (boards, pieces, masks, old_log_probs, advantages, returns))
    _, new_log_probs, entropy, values = network.get_action_and_value(boards, pieces, masks, actions)
    ratio = torch.exp(new_log_probs - old_log_probs)
    surr1 = ratio * advantages
    surr2 = torch.clamp(ratio, 1 - cfg.clip_epsilon, 1 + cfg.clip_epsilon) * advantages
    policy_loss = -torch.min(surr1, surr2).mean()
    value_loss = F.mse_loss(values, returns)
    entropy_loss = -entropy.mean()
    loss = policy_loss + cfg.value_coef * value_loss + cfg.entropy_coef * entropy_loss
    return policy_loss, value_loss, entropy, loss, ratio


def clipped_grads(network: ReferenceNetwork, batch, cfg) -> Dict[str, torch.Tensor]:
    """The minibatch's gradients after clip_grad_norm_(max_grad_norm)
    (ppo.py:395-400) in the network's own dtype (tests run it in float64 as
    the ground truth that fp32 implementations are measured against)."""
    network.zero_grad(set_to_none=True)
    minibatch_loss(network, batch, cfg)[3].backward()
    nn.utils.clip_grad_norm_(network.parameters(), cfg.max_grad_norm)
    return {n: p.grad.detach().clone() for n, p in network.named_parameters() if p.grad is not None}


def ppo_update(network: ReferenceNetwork, optimizer: torch.optim.Optimizer, buf: Dict[str, np.ndarray],
               last_values: np.ndarray, cfg, permutation: Callable[[int], np.ndarray],
               before_step: Optional[Callable[[int], None]] = None,
               after_step: Optional[Callable[..., None]] = None):
    """PPOAgent.update (ppo.py:330-423) on a CPU float32 buffer in the
    reference's layout (boards, pieces, action_masks f32; actions i64;
    log_probs, rewards, dones, values f32; all [T, N, ...]).  ``cfg`` carries
    the PPOConfig fields; ``permutation(total)`` supplies each epoch's
    minibatch order; ``before_step(k)`` / ``after_step(k, stats)`` run around
    optimizer step k (tests load another implementation's state there, so each
    step is compared from identical weights; after_step also gets the
    minibatch).  Returns (metric means, per-minibatch statistics [n, 6],
    advantages, returns)."""
    adv, ret = gae(buf["rewards"], buf["values"], buf["dones"], last_values, cfg.gamma, cfg.gae_lambda)
    buf = dict(buf, advantages=adv, returns=ret)
    T, N = buf["rewards"].shape
    rows: List[List[float]] = []
    for _ in range(cfg.num_epochs):
        for batch in get_samples(buf, cfg.batch_size, permutation(T * N)):
            if before_step is not None:
                before_step(len(rows))
            policy_loss, value_loss, entropy, loss, ratio = minibatch_loss(network, batch, cfg)
            optimizer.zero_grad()
            loss.backward()
            nn.utils.clip_grad_norm_(network.parameters(), cfg.max_grad_norm)
            optimizer.step()
            with torch.no_grad():
                approx_kl = ((ratio - 1) - torch.log(ratio)).mean()
                clip_fraction = ((ratio - 1).abs() > cfg.clip_epsilon).float().mean()
            rows.append([policy_loss.item(), value_loss.item(), entropy.mean().item(), loss.item(),
                         approx_kl.item(), clip_fraction.item()])
            if after_step is not None:
                after_step(len(rows) - 1, rows[-1], batch)
    per = np.array(rows, dtype=np.float64).reshape(-1, 6)
    means = {k: sum(r[j] for r in rows) / max(len(rows), 1) for j, k in enumerate(STAT_KEYS)}  # ppo.py:408-423
    return means, per, adv, ret
