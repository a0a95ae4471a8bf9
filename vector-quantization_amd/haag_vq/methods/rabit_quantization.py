"""1-bit RaBitQ on the MI355X.

Drop-in for the reference's ``RaBitQuantizer``
(/root/reference/src/haag_vq/methods/rabit_quantization.py:9-40), which wraps
``faiss.RaBitQuantizer(D, metric)`` (train is a no-op: no centroid, no rotation).  Codes
follow faiss' layout: ceil(D/8) sign bytes (LSB-first) + two f32 factors; encode and decode
are ``mivq_rabitq_encode`` / ``mivq_rabitq_decode``.  Callers detect this class by name
(``type(model).__name__ == "RaBitQuantizer"``, faiss_export.py:37-38), so the name is kept.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _arrays, _native
from ..utils.faiss_utils import MetricType
from .base_quantizer import BaseQuantizer


class RaBitQHandle:
    """Stands where the reference keeps ``faiss.RaBitQuantizer`` (``model.rabitq``)."""

    def __init__(self, owner: "RaBitQuantizer", d: int) -> None:
        self._owner = owner
        self.d = d
        self.metric_type = int(owner.metric_type)
        self.code_size = _native.rabitq_code_size(d)

    def compute_codes(self, x):
        return self._owner.compress(x)

    def decode(self, codes):
        return self._owner.decompress(codes)


class RaBitQuantizer(BaseQuantizer):
    def __init__(self, metric_type: MetricType = MetricType.L2):
        """RaBitQ (Gao & Long, SIGMOD 2024), 1 bit per dimension."""
        self.metric_type = metric_type
        self.rabitq: RaBitQHandle | None = None

    def fit(self, X):
        N, D = X.shape
        if int(self.metric_type) not in (int(MetricType.L2), int(MetricType.INNER_PRODUCT)):
            raise RuntimeError(f"RaBitQuantizer supports L2 / INNER_PRODUCT only, got {self.metric_type!r}")
        self.rabitq = RaBitQHandle(self, int(D))

    def _require(self, what):
        if self.rabitq is None:
            raise RuntimeError(f"RaBitQuantizer must be fitted before {what}().")

    def compress(self, X):
        self._require("compress")
        m = int(self.metric_type)
        if _arrays.is_tensor(X):
            return _native.rabitq_encode(_arrays.to_device(X), None, m)
        X = np.asarray(X, dtype=np.float32)
        n, d = X.shape
        out = np.empty((n, _native.rabitq_code_size(d)), dtype=np.uint8)
        for s, e in _arrays.row_chunks(n, d * 4):
            out[s:e] = _arrays.to_host(_native.rabitq_encode(_arrays.to_device(X[s:e]), None, m))
        return out

    def decompress(self, compressed):
        self._require("decompress")
        d = self.rabitq.d
        if _arrays.is_tensor(compressed):
            return _native.rabitq_decode(_arrays.to_device(compressed, torch.uint8), d, None)
        compressed = np.asarray(compressed)
        n = compressed.shape[0]
        out = np.empty((n, d), dtype=np.float32)
        for s, e in _arrays.row_chunks(n, d * 4):
            out[s:e] = _arrays.to_host(_native.rabitq_decode(_arrays.to_device(compressed[s:e], torch.uint8), d, None))
        return out

    def get_compression_ratio(self, X):
        D = int(X.shape[1])
        return float(D * 4 / int(self.rabitq.code_size))
