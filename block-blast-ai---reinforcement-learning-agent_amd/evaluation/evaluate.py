"""Evaluation of a trained agent (reference scripts/evaluate.py:23-90 and its
CLI 119-184).

The reference plays ``num_episodes`` games one after another on a single
``BlockBlastEnv`` re-seeded ``seed + episode``.  Episodes are independent, so
here they run side by side: one device env per episode (seeded
``seed + episode``, no auto-reset) stepped in lockstep, the policy evaluated
for all unfinished games in one forward pass, each game's statistics latched
at its termination.  With ``deterministic=True`` (argmax) and the agent in
eval mode this gives the same per-episode results as the sequential loop.
``render=True`` uses the sequential single-env path so games can be shown.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import Any, Dict

import numpy as np
import torch


def _summary(scores, lengths, lines, combos) -> Dict[str, Any]:
    return {
        "num_episodes": len(scores), "mean_score": np.mean(scores), "std_score": np.std(scores),
        "min_score": np.min(scores), "max_score": np.max(scores), "median_score": np.median(scores),
        "mean_length": np.mean(lengths), "std_length": np.std(lengths),
        "mean_lines_cleared": np.mean(lines), "mean_max_combo": np.mean(combos),
        "scores": list(scores), "lengths": list(lengths),
    }


def _evaluate_sequential(agent, num_episodes: int, deterministic: bool, render: bool, seed: int,
                         record_actions: bool = False):
    from environment.block_blast_env import BlockBlastEnv

    env = BlockBlastEnv(render_mode="human" if render else None, seed=seed)
    scores, lengths, lines, combos, actions = [], [], [], [], []
    for ep in range(num_episodes):
        obs, info = env.reset(seed=seed + ep)
        done, n, score = False, 0, 0
        actions.append([])
        while not done:
            action, _ = agent.select_action(obs, deterministic=deterministic)
            actions[-1].append(int(action))
            obs, _, terminated, truncated, info = env.step(action)
            done = terminated or truncated
            n += 1
            if render:
                env.render()
            if done:
                score = info.get("score", 0)
        scores.append(score)
        lengths.append(n)
        lines.append(info.get("lines_cleared", 0))
        combos.append(info.get("max_combo", 0))
    env.close()
    res = _summary(scores, lengths, lines, combos)
    if record_actions:
        res["actions"] = actions
    return res


def evaluate_agent(agent, num_episodes: int = 100, deterministic: bool = True, render: bool = False,
                   seed: int = 42, max_moves: int = 100_000, record_actions: bool = False) -> Dict[str, Any]:
    """evaluate.py:23-90 (same keys in the returned dict).  record_actions: also return every episode's
    action sequence under "actions" (for replaying the games elsewhere, e.g. through the oracle)."""
    agent.eval()
    if render:
        return _evaluate_sequential(agent, num_episodes, deterministic, render, seed, record_actions)
    from runtime.device_env import DeviceEnvBatch

    dev = agent.device
    n = num_episodes
    env = DeviceEnvBatch(n, [seed + e for e in range(n)], autoreset=False, device=dev)
    env.reset()
    x = torch.zeros((n, 4, 8, 8), dtype=torch.float32, device=dev)
    mb = torch.zeros((n, 3), dtype=torch.int64, device=dev)
    act = torch.zeros(n, dtype=torch.int32, device=dev)
    alive = torch.ones(n, dtype=torch.bool, device=dev)
    length = torch.zeros(n, dtype=torch.int64, device=dev)
    rec = torch.zeros((n, 4), dtype=torch.int64, device=dev)  # score, lines, max_combo, done
    info64 = env.info.view(torch.int64).view(n, 7)
    info32 = env.info.view(torch.int32).view(n, 14)
    log = []
    for step in range(max_moves):
        env.obs(x=x, mask_bits=mb)
        a, _, _ = agent.act_device(x, mb, deterministic=deterministic)
        act.copy_(a)
        if record_actions:
            log.append(act.clone())
        env.step(act, want_info=True)
        length += alive.long()
        term = env.terminated.bool() & alive
        rec[:, 0] = torch.where(term, info64[:, 0], rec[:, 0])
        rec[:, 1] = torch.where(term, info32[:, 7].long(), rec[:, 1])
        rec[:, 2] = torch.where(term, info32[:, 8].long(), rec[:, 2])
        alive &= ~term
        if step % 16 == 15 and not bool(alive.any()):
            break
    out = rec.cpu().numpy()
    lengths = length.cpu().numpy()
    env.close()
    res = _summary(out[:, 0].tolist(), lengths.tolist(), out[:, 1].tolist(), out[:, 2].tolist())
    if record_actions:
        acts = torch.stack(log).cpu().numpy() if log else np.zeros((0, n), np.int32)
        res["actions"] = [acts[:int(lengths[e]), e].tolist() for e in range(n)]
    return res


def print_results(results: Dict[str, Any]) -> None:
    """evaluate.py:93-117."""
    print("\n" + "=" * 60)
    print("EVALUATION RESULTS")
    print("=" * 60)
    print(f"Episodes: {results['num_episodes']}")
    print()
    print("Score Statistics:")
    print(f"  Mean:   {results['mean_score']:.1f} ± {results['std_score']:.1f}")
    print(f"  Median: {results['median_score']:.1f}")
    print(f"  Min:    {results['min_score']:.1f}")
    print(f"  Max:    {results['max_score']:.1f}")
    print()
    print("Game Statistics:")
    print(f"  Mean length: {results['mean_length']:.1f} ± {results['std_length']:.1f}")
    print(f"  Mean lines cleared: {results['mean_lines_cleared']:.1f}")
    print(f"  Mean max combo: {results['mean_max_combo']:.1f}")
    print("=" * 60)
    print("\nScore Percentiles:")
    for p in (10, 25, 50, 75, 90, 95, 99):
        print(f"  {p}th: {np.percentile(results['scores'], p):.1f}")


def main() -> None:
    """evaluate.py:119-184 (same flags)."""
    ap = argparse.ArgumentParser(description="Evaluate Block Blast AI")
    ap.add_argument("--checkpoint", type=str, required=True)
    ap.add_argument("--episodes", type=int, default=100)
    ap.add_argument("--deterministic", action="store_true")
    ap.add_argument("--render", action="store_true")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--output", type=str, default=None)
    args = ap.parse_args()
    if not os.path.exists(args.checkpoint):
        print(f"Checkpoint not found: {args.checkpoint}")
        sys.exit(1)
    from agents.ppo import PPOAgent
    from utils.device import get_device

    agent = PPOAgent(device=get_device())
    agent.load(args.checkpoint)
    print(f"Loaded model from {args.checkpoint}")
    res = evaluate_agent(agent, num_episodes=args.episodes, deterministic=args.deterministic, render=args.render,
                         seed=args.seed)
    print_results(res)
    if args.output:
        with open(args.output, "w") as f:
            json.dump({k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in res.items()}, f, indent=2,
                      default=float)
        print(f"\nResults saved to {args.output}")


if __name__ == "__main__":
    main()
