#!/usr/bin/env python3
"""CLI: python evaluate.py --checkpoint checkpoints/best.pt [--episodes 100] [--deterministic] [--seed 42]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

from evaluation.evaluate import main  # noqa: E402

if __name__ == "__main__":
    main()
