"""Search-index contract — same interface as
/root/reference/src/haag_vq/methods/base_search_index.py:21-89."""

from __future__ import annotations

from abc import ABC, abstractmethod
from pathlib import Path
from typing import Literal, Optional, Tuple

import numpy as np


class BaseSearchIndex(ABC):
    """fit / search / search_with_scores / memory_footprint / save / load."""

    @abstractmethod
    def fit(self, X: np.ndarray, metric: Literal["l2", "ip"] = "l2") -> None:
        """Learn the index from X (N, D); search() and memory_footprint() valid afterwards."""

    @abstractmethod
    def search(self, Q: np.ndarray, k: int) -> np.ndarray:
        """(nq, k) uint32 approximate nearest-neighbour ids."""

    @abstractmethod
    def search_with_scores(self, Q: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
        """(ids uint32, distances float32), both (nq, k): squared L2 ascending, or IP descending."""

    @abstractmethod
    def memory_footprint(self) -> int:
        """Bytes of encoded data plus auxiliary structures."""

    @abstractmethod
    def save(self, path: str | Path) -> None:
        """Persist the index."""

    @abstractmethod
    def load(self, path: str | Path) -> None:
        """Restore the index."""

    def reconstruction_mse(self, X: np.ndarray, sample_ids: Optional[np.ndarray] = None) -> Optional[float]:
        """Mean per-element reconstruction MSE, or None when unsupported."""
        return None
