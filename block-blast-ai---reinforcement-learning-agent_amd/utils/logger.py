"""Training metric sinks with the reference's file formats and semantics
(src/utils/logger.py): a JSONL record per ``log`` call, a console dump, a
``{name}_summary.json`` of per-metric mean/std/min/max/last, an optional
TensorBoard writer, and a rolling-window ``MetricsTracker``.

Under torch.distributed only rank 0 should construct writers (the trainer
passes ``enabled=False`` elsewhere).
"""
from __future__ import annotations

import json
import math
import time
from collections import defaultdict, deque
from datetime import datetime
from pathlib import Path
from typing import Any, Deque, Dict, List, Optional

import numpy as np


def _plain(v: Any) -> Any:
    """logger.py:13-25: numpy / torch scalars and arrays -> JSON types."""
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.generic):
        return v.item()
    if hasattr(v, "item") and callable(v.item) and getattr(v, "numel", lambda: 0)() == 1:
        return v.item()
    return v


class Logger:
    """logger.py:28-131."""

    def __init__(self, log_dir: str, name: str = "training", enabled: bool = True):
        self.log_dir = Path(log_dir)
        self.name = name
        self.enabled = enabled
        self.start_time = time.time()
        self.step = 0
        self.metrics_history: Dict[str, List[float]] = defaultdict(list)
        stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
        self.log_file = self.log_dir / f"{name}_{stamp}.jsonl"
        if enabled:
            self.log_dir.mkdir(parents=True, exist_ok=True)

    def log(self, metrics: Dict[str, Any], step: Optional[int] = None) -> None:
        self.step = self.step + 1 if step is None else step
        for k, v in metrics.items():
            if isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool):
                self.metrics_history[k].append(float(v))
        if not self.enabled:
            return
        rec = {"step": self.step, "time": time.time() - self.start_time,
               "timestamp": datetime.now().isoformat(), **metrics}
        with open(self.log_file, "a") as f:
            f.write(json.dumps(_plain(rec)) + "\n")

    def get_recent(self, metric: str, n: int = 100) -> List[float]:
        return self.metrics_history[metric][-n:]

    def get_mean(self, metric: str, n: int = 100) -> float:
        r = self.get_recent(metric, n)
        return float(np.mean(r)) if r else 0.0

    def print_metrics(self, metrics: Dict[str, Any]) -> None:
        if not self.enabled:
            return
        e = int(time.time() - self.start_time)
        print(f"\n[Step {self.step:,}] [{e // 3600:02d}:{e % 3600 // 60:02d}:{e % 60:02d}]")
        for k, v in metrics.items():
            print(f"  {k}: {v:.4f}" if isinstance(v, float) else f"  {k}: {v}")

    def save_summary(self) -> None:
        if not self.enabled:
            return
        out = {"name": self.name, "total_steps": self.step, "total_time": time.time() - self.start_time,
               "metrics": {}}
        for k, vals in self.metrics_history.items():
            a = np.asarray(vals, dtype=np.float64)
            out["metrics"][k] = {"mean": float(a.mean()), "std": float(a.std()), "min": float(a.min()),
                                 "max": float(a.max()), "last": float(a[-1])}
        self.log_dir.mkdir(parents=True, exist_ok=True)
        with open(self.log_dir / f"{self.name}_summary.json", "w") as f:
            json.dump(out, f, indent=2)


class TensorBoardLogger:
    """logger.py:134-219; a silent no-op when tensorboard is not importable."""

    def __init__(self, log_dir: str, name: str = "training", enabled: bool = True):
        self.writer = None
        if not enabled:
            return
        try:
            from torch.utils.tensorboard import SummaryWriter
        except Exception:  # tensorboard package absent
            return
        self.writer = SummaryWriter(str(Path(log_dir) / "tensorboard" / name))

    def log_scalar(self, tag: str, value: float, step: Optional[int] = None) -> None:
        if self.writer is not None:
            self.writer.add_scalar(tag, value, step)

    def log_scalars(self, main_tag: str, values: Dict[str, float], step: Optional[int] = None) -> None:
        if self.writer is not None:
            self.writer.add_scalars(main_tag, values, step)

    def log_histogram(self, tag: str, values, step: Optional[int] = None) -> None:
        if self.writer is not None:
            self.writer.add_histogram(tag, values, step)

    def log_metrics(self, metrics: Dict[str, float], step: Optional[int] = None) -> None:
        for k, v in metrics.items():
            if isinstance(v, (int, float)) and math.isfinite(float(v)):
                self.log_scalar(k, v, step)

    def close(self) -> None:
        if self.writer is not None:
            self.writer.close()


class MetricsTracker:
    """logger.py:222-284: rolling window of the last ``window_size`` values."""

    def __init__(self, window_size: int = 100):
        self.window_size = window_size
        self.metrics: Dict[str, Deque[float]] = defaultdict(lambda: deque(maxlen=self.window_size))

    def add(self, name: str, value: float) -> None:
        self.metrics[name].append(value)

    def extend(self, name: str, values) -> None:
        self.metrics[name].extend(values)

    def _v(self, name: str):
        return list(self.metrics.get(name, ()))

    def get_mean(self, name: str) -> float:
        v = self._v(name)
        return float(np.mean(v)) if v else 0.0

    def get_std(self, name: str) -> float:
        v = self._v(name)
        return float(np.std(v)) if v else 0.0

    def get_min(self, name: str) -> float:
        v = self._v(name)
        return float(np.min(v)) if v else 0.0

    def get_max(self, name: str) -> float:
        v = self._v(name)
        return float(np.max(v)) if v else 0.0

    def get_last(self, name: str) -> float:
        v = self._v(name)
        return v[-1] if v else 0.0

    def get_summary(self, name: str) -> Dict[str, float]:
        return {"mean": self.get_mean(name), "std": self.get_std(name), "min": self.get_min(name),
                "max": self.get_max(name), "last": self.get_last(name)}

    def get_all_summaries(self) -> Dict[str, Dict[str, float]]:
        return {k: self.get_summary(k) for k in self.metrics}

    def reset(self) -> None:
        self.metrics.clear()
