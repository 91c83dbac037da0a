#!/usr/bin/env python3
"""Training launcher with the reference CLI (run_train.py:47-150):
``python run_train.py [--config config/default.yaml] [--resume ckpt.pt] [--seed 42]``.

Multi-GPU: ``python -m torch.distributed.run --nproc-per-node N --master-addr
127.0.0.1 run_train.py --config ...`` (one process per MI355X, RCCL).
"""
import argparse
import os
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))


def main() -> None:
    ap = argparse.ArgumentParser(description="Block Blast AI - Terminal Training")
    ap.add_argument("--config", type=str, default="config/default.yaml")
    ap.add_argument("--resume", type=str, default=None)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--max-updates", type=int, default=None, help="stop after this many PPO updates")
    args = ap.parse_args()

    from training.trainer import DEFAULT_CONFIG, load_config, train

    path = Path(args.config)
    if not path.exists() and not path.is_absolute():
        path = HERE / args.config
    if path.exists():
        config = load_config(str(path))
        print(f"Loaded config from: {path}")
    else:
        print(f"Config file not found: {args.config}")
        print("Using default configuration")
        config = DEFAULT_CONFIG
    t = config.get("training", {})
    if int(os.environ.get("RANK", "0")) == 0:
        print("Training Configuration:")
        print(f"  Total timesteps: {t.get('total_timesteps', 10_000_000):,}")
        print(f"  Parallel envs: {t.get('num_envs', 64)}")
        print(f"  Batch size: {t.get('batch_size', 2048)}")
        print(f"  Rollout steps: {t.get('rollout_steps', 128)}")
        print()
    try:
        train(config, resume_path=args.resume, seed=args.seed, max_updates=args.max_updates)
    except KeyboardInterrupt:
        print("\nTraining interrupted by user")


if __name__ == "__main__":
    main()
