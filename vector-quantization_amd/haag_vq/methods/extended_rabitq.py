"""Multi-bit ("Extended") RaBitQ on the MI355X.

Drop-in for the reference's ``ExtendedRaBitQuantizer``
(/root/reference/src/haag_vq/methods/extended_rabitq.py:47-204), the quantizer the registry's
``rabitq`` method builds (method_registry_saq.py:45-48).  Model state is computed exactly as the
reference does (global fp64 mean, QR of a seeded Gaussian matrix, 1-D Lloyd levels on an N(0,1)
sample — host-side, data independent except the mean); the per-row work runs on the device:
``mivq_extrabitq_normalize`` -> fp64 GEMM (o . P) -> ``mivq_extrabitq_quantize`` (searchsorted,
rescale factor t, MSB-first packing) and the mirror image for decode.  Code rows are
``ceil(D*B/8) + 8`` bytes (indices ++ f32 norm ++ f32 t) and decode row-independently.

Parity: fp64 throughout; the GEMM's summation order differs from numpy/OpenBLAS, so an index
can differ only where s lies within rounding distance of a level midpoint (each such index is
checked to be a midpoint tie against the reference's fixtures in
tests/test_pinning_gpu.py::test_extrabitq_mismatches_are_midpoint_ties), and the decoded
vectors agree to ~1e-12 relative.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _arrays, _native
from .base_quantizer import BaseQuantizer


def _lloyd_1d_normal(num_levels: int, seed: int, n_samples: int = 200_000, max_iter: int = 100,
                     tol: float = 1e-7) -> np.ndarray:
    """Gaussian-optimal scalar codebook by 1-D Lloyd (extended_rabitq.py:6-44)."""
    rng = np.random.default_rng(seed)
    samples = rng.standard_normal(n_samples)
    levels = np.quantile(samples, (np.arange(num_levels) + 0.5) / num_levels)
    for _ in range(max_iter):
        idx = np.searchsorted(0.5 * (levels[:-1] + levels[1:]), samples)
        new = levels.copy()
        for k in range(num_levels):
            sel = idx == k
            if np.any(sel):
                new[k] = samples[sel].mean()
        new.sort()
        shift = float(np.max(np.abs(new - levels)))
        levels = new
        if shift < tol:
            break
    return levels.astype(np.float64)


class ExtendedRaBitQuantizer(BaseQuantizer):
    def __init__(self, num_bits: int = 4, seed: int = 0):
        if num_bits < 1 or num_bits > 8:
            raise ValueError("num_bits must be in [1, 8]")
        self.num_bits = int(num_bits)
        self.seed = int(seed)
        self.c: np.ndarray | None = None
        self.P: np.ndarray | None = None
        self.levels: np.ndarray | None = None
        self.D: int | None = None
        self._eps = 1e-12
        self._dev = None

    def fit(self, X) -> None:
        if _arrays.is_tensor(X):
            self.D = int(X.shape[1])
            self.c = _arrays.to_host(X.to(torch.float64).mean(dim=0))
        else:
            X = np.asarray(X)
            self.D = int(X.shape[1])
            self.c = X.mean(axis=0).astype(np.float64)
        rng = np.random.default_rng(self.seed)
        Q, _ = np.linalg.qr(rng.standard_normal((self.D, self.D)))
        self.P = Q.astype(np.float64)
        self.levels = _lloyd_1d_normal(2 ** self.num_bits, seed=self.seed)
        self._dev = None

    @property
    def _index_bytes(self) -> int:
        return (self.D * self.num_bits + 7) // 8

    @property
    def code_size(self) -> int:
        return self._index_bytes + 8

    def _state(self):
        if self._dev is None:
            dev = _arrays.device()
            self._dev = tuple(torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(dev)
                              for a in (self.c, self.P, self.levels))
        return self._dev

    def compress(self, X):
        if self.P is None:
            raise RuntimeError("Quantizer must be fit before compress().")
        c, P, lv = self._state()
        if _arrays.is_tensor(X):
            if X.shape[1] != self.D:
                raise ValueError(f"compress() got D={X.shape[1]}, but fit() saw D={self.D}")
            xt = X if X.dtype in (torch.float32, torch.float64) else X.to(torch.float64)
            return _native.extrabitq_encode(_arrays.to_device(xt, xt.dtype), c, P, lv, self.num_bits)
        X = np.asarray(X)
        if X.shape[1] != self.D:
            raise ValueError(f"compress() got D={X.shape[1]}, but fit() saw D={self.D}")
        dt = torch.float64 if X.dtype == np.float64 else torch.float32
        out = np.empty((X.shape[0], self.code_size), np.uint8)
        for s, e in _arrays.row_chunks(X.shape[0], self.D * 24):
            out[s:e] = _arrays.to_host(_native.extrabitq_encode(_arrays.to_device(X[s:e], dt), c, P, lv, self.num_bits))
        return out

    def decompress(self, codes):
        if self.P is None:
            raise RuntimeError("Quantizer must be fit before decompress().")
        c, P, lv = self._state()
        if _arrays.is_tensor(codes):
            return _native.extrabitq_decode(_arrays.to_device(codes, torch.uint8), c, P, lv, self.num_bits)
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        out = np.empty((codes.shape[0], self.D), np.float32)
        for s, e in _arrays.row_chunks(codes.shape[0], self.D * 24):
            out[s:e] = _arrays.to_host(_native.extrabitq_decode(_arrays.to_device(codes[s:e], torch.uint8),
                                                                c, P, lv, self.num_bits))
        return out

    def get_compression_ratio(self, X) -> float:
        return float(int(X.shape[1]) * 4 / self.code_size)
