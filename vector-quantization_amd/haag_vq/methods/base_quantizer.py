"""The quantizer plugin contract.

Same interface as the reference's ``BaseQuantizer``
(/root/reference/src/haag_vq/methods/base_quantizer.py:8-91): ``fit`` / ``compress`` /
``decompress`` plus the codebook export helper.  Implementations in this package run
their hot path on the MI355X through libmivq.so.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from pathlib import Path
from typing import Any, Dict, Optional, Union

import numpy as np


class BaseQuantizer(ABC):
    """Abstract quantizer: learn parameters (fit), encode (compress), decode (decompress)."""

    @abstractmethod
    def fit(self, X: np.ndarray) -> None:
        """Learn quantization parameters from training data X of shape (N, D)."""

    @abstractmethod
    def compress(self, X: np.ndarray) -> np.ndarray:
        """Encode X (N, D) into codes (one row per vector)."""

    @abstractmethod
    def decompress(self, codes: np.ndarray) -> np.ndarray:
        """Reconstruct approximations (N, D) from codes."""

    def save_codebooks(
        self,
        *,
        codes: Optional[np.ndarray] = None,
        output_dir: Optional[Union[str, Path]] = None,
        codebook_filename: Optional[str] = None,
        codes_filename: Optional[str] = None,
    ) -> Dict[str, Any]:
        """Write the codebook (.fvecs) and optional codes (.ivecs) — base_quantizer.py:53-91."""
        from haag_vq.utils.faiss_export import export_codebook

        target = Path(output_dir) if output_dir is not None else Path.cwd() / "codebooks"
        target.mkdir(parents=True, exist_ok=True)
        prefix = type(self).__name__.lower()
        return export_codebook(
            self,
            target,
            codes=codes,
            codebook_filename=codebook_filename or f"{prefix}_codebook.fvecs",
            codes_filename=codes_filename or f"{prefix}_codes.ivecs",
        )
