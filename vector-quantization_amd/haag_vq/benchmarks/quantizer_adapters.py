"""Quantizer protocol + adapter for the benchmark study.

Same contract as /root/reference/src/haag_vq/benchmarks/quantizer_adapters.py:17-59: the
adapter encodes the whole database at fit, reconstructs by global id, and reports stored
bytes including the 4-byte exact-norm side channel.  Codes stay resident on the device.
(The SAQ-engine adapter of the reference is out of scope.)
"""

from __future__ import annotations

from typing import Optional, Protocol, runtime_checkable

import numpy as np
import torch

from haag_vq import _arrays
from haag_vq.methods.base_quantizer import BaseQuantizer

NORM_SIDECHANNEL_BYTES = 4


@runtime_checkable
class Quantizer(Protocol):
    def fit(self, X: np.ndarray) -> None: ...
    def reconstruct(self, ids: np.ndarray) -> np.ndarray: ...
    def code_bytes(self) -> int: ...


class FaissQuantizerAdapter:
    """Adapts a BaseQuantizer (PQ / OPQ / SQ / RaBitQ / ExtRaBitQ) to the Quantizer protocol."""

    def __init__(self, quantizer: BaseQuantizer) -> None:
        self._q = quantizer
        self._codes: Optional[torch.Tensor] = None
        self._n = 0

    @property
    def quantizer(self) -> BaseQuantizer:
        return self._q

    @property
    def codes(self) -> torch.Tensor:
        return self._codes

    def fit(self, X) -> None:
        Xd = _arrays.to_device(X, torch.float32)
        self._q.fit(Xd)
        codes = self._q.compress(Xd)  # may raise; leave prior state intact
        self._codes = codes if _arrays.is_tensor(codes) else torch.from_numpy(np.asarray(codes)).to(Xd.device)
        self._n = Xd.shape[0]

    def reconstruct(self, ids) -> np.ndarray:
        if self._codes is None:
            raise RuntimeError("FaissQuantizerAdapter.reconstruct() before fit()")
        ids = np.asarray(ids, dtype=np.int64)
        if np.any(ids < 0):
            raise ValueError("reconstruct(): negative ids are not allowed")
        sel = self._codes[torch.from_numpy(ids).to(self._codes.device)].contiguous()
        rec = self._q.decompress(sel)
        if _arrays.is_tensor(rec):
            rec = _arrays.to_host(rec)
        return np.asarray(rec, dtype=np.float32)

    def code_bytes(self) -> int:
        if self._codes is None:
            raise RuntimeError("FaissQuantizerAdapter.code_bytes() before fit()")
        return int(self._codes.numel() * self._codes.element_size()) + self._n * NORM_SIDECHANNEL_BYTES
