#!/usr/bin/env python3
"""BASELINE config 1 on the host CPU: one PPO iteration of the reference's
default.yaml path -- 64 envs stepped sequentially (the oracle's cell-loop
port of wrappers.py / block_blast_env.py / engine.py, as the reference loops
in Python, wrappers.py:93), T = 128 rollout steps with a train-mode CNN
forward per step and a torch Categorical sample (scripts/train.py:173-203,
ppo.py:291-319), then GAE (ppo.py:141-169) and 10 epochs x 4 minibatches of
2048 (ppo.py:330-423: clipped surrogate, value MSE, entropy, grad-norm 0.5,
Adam eps 1e-5).  SURVEY.md 8(d) C1: env-steps/s = 8192 / (rollout + update),
rollout-only reported beside it; torch intra-op threads = all host cores.

This is the reference's CPU path restated (the reference itself cannot be run
here); it is a reported baseline for BASELINE config 3, not
the thing measured by bench.py.  Prints one JSON line.
"""
import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch.distributions import Categorical  # noqa: E402


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--rollout", type=int, default=128)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--threads", type=int, default=0, help="torch intra-op threads (0: all host cores)")
    args = ap.parse_args()

    from agents.ppo import PPOConfig, ppo_loss_torch
    from models.network import BlockBlastNetwork
    from oracle import bb_game as O
    from oracle import bb_ppo as OP

    cores = os.cpu_count() or 1
    torch.set_num_threads(args.threads or cores)
    torch.manual_seed(0)
    np.random.seed(0)
    cfg = PPOConfig(batch_size=args.batch, num_epochs=args.epochs)
    net = BlockBlastNetwork()
    net.train()  # rollouts run in train mode too (scripts/train.py:122)
    opt = torch.optim.Adam(net.parameters(), lr=cfg.learning_rate, eps=1e-5)
    n, T = args.envs, args.rollout
    vec = O.VecEnv(n, seed=42)
    obs, _ = vec.reset()

    boards = np.zeros((T, n, 8, 8), np.float32)
    pieces = np.zeros((T, n, 3, 8, 8), np.float32)
    masks = np.zeros((T, n, 192), np.float32)
    actions = np.zeros((T, n), np.int64)
    logps = np.zeros((T, n), np.float32)
    rewards = np.zeros((T, n), np.float32)
    dones = np.zeros((T, n), np.float32)
    values = np.zeros((T, n), np.float32)

    t0 = time.perf_counter()
    for t in range(T):  # scripts/train.py:173-203
        b = torch.from_numpy(np.asarray(obs["board"], np.float32))
        p = torch.from_numpy(np.asarray(obs["pieces"], np.float32))
        m = torch.from_numpy(np.asarray(obs["action_mask"], np.float32))
        with torch.no_grad():
            logits, v = net.raw(BlockBlastNetwork.stack_input(b, p))
            masked = logits + torch.where(m.bool(), torch.zeros_like(logits), torch.full_like(logits, float("-inf")))
            dist = Categorical(probs=F.softmax(masked, dim=-1))
            a = dist.sample()
            lp = dist.log_prob(a)
        boards[t], pieces[t], masks[t] = b.numpy(), p.numpy(), m.numpy()
        actions[t], logps[t], values[t] = a.numpy(), lp.numpy(), v.numpy()
        obs, r, term, _, _ = vec.step(a.numpy())
        rewards[t], dones[t] = r, term.astype(np.float32)
    with torch.no_grad():
        last = net.raw(BlockBlastNetwork.stack_input(torch.from_numpy(np.asarray(obs["board"], np.float32)),
                                                     torch.from_numpy(np.asarray(obs["pieces"], np.float32))))[1]
    t_roll = time.perf_counter() - t0

    t0 = time.perf_counter()
    adv, ret = OP.gae(rewards, values, dones, last.numpy().astype(np.float32), np.float32(cfg.gamma),
                      np.float32(cfg.gae_lambda))
    total = T * n
    adv_n = OP.normalize_advantages(adv).astype(np.float32)
    X = BlockBlastNetwork.stack_input(torch.from_numpy(boards.reshape(total, 8, 8)),
                                      torch.from_numpy(pieces.reshape(total, 3, 8, 8)))
    Mk = torch.from_numpy(masks.reshape(total, 192))
    A = torch.from_numpy(actions.reshape(total))
    LP = torch.from_numpy(logps.reshape(total))
    ADV = torch.from_numpy(adv_n)
    RET = torch.from_numpy(ret.reshape(total).astype(np.float32))
    steps = 0
    for _ in range(cfg.num_epochs):  # ppo.py:347-423
        perm = torch.from_numpy(np.random.permutation(total))
        for s in range(0, total, cfg.batch_size):
            idx = perm[s:s + cfg.batch_size]
            logits, v = net.raw(X[idx])
            loss, _stats = ppo_loss_torch(logits, v, Mk[idx], A[idx], LP[idx], ADV[idx], RET[idx], cfg)
            opt.zero_grad()
            loss.backward()
            nn.utils.clip_grad_norm_(net.parameters(), cfg.max_grad_norm)
            opt.step()
            steps += 1
    t_upd = time.perf_counter() - t0
    print(json.dumps({
        "workload": "BASELINE config 1: default.yaml PPO iteration on the host CPU (reference path restated)",
        "envs": n, "rollout_steps": T, "batch": cfg.batch_size, "epochs": cfg.num_epochs, "optimizer_steps": steps,
        "rollout_s": round(t_roll, 3), "update_s": round(t_upd, 3),
        "rollout_env_steps_per_s": round(total / t_roll, 1),
        "ppo_env_steps_per_s": round(total / (t_roll + t_upd), 1),
        "nproc": cores, "torch_threads": torch.get_num_threads(), "cpu_model": cpu_model(),
        "env": "oracle/bb_game.py VecEnv (cell loops, one Python thread)", "compute_dtype": "fp32",
    }))


if __name__ == "__main__":
    main()
