"""Agent interface (reference src/agents/base.py:10-87)."""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Dict, Tuple

import torch


class BaseAgent(ABC):
    def __init__(self, device: torch.device):
        self.device = device
        self.training = True

    @abstractmethod
    def select_action(self, observation: Dict[str, Any], deterministic: bool = False) -> Tuple[int, Dict[str, Any]]:
        ...

    @abstractmethod
    def update(self, *args, **kwargs) -> Dict[str, float]:
        ...

    @abstractmethod
    def save(self, path: str) -> None:
        ...

    @abstractmethod
    def load(self, path: str) -> None:
        ...

    def train(self) -> None:
        self.training = True

    def eval(self) -> None:
        self.training = False

    def to(self, device: torch.device) -> "BaseAgent":
        self.device = device
        return self
