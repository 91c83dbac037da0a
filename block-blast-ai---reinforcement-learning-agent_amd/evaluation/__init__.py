"""Agent evaluation (reference scripts/evaluate.py)."""
from .evaluate import evaluate_agent, print_results  # noqa: F401
