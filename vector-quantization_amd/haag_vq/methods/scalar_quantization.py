"""Scalar quantization (4 / 8 / 16 bit) on the MI355X.

Drop-in for the reference's ``ScalarQuantizer``
(/root/reference/src/haag_vq/methods/scalar_quantization.py:6-100): per-dimension min/max
fit, ``round(((x - min) / (max - min + 1e-8)) * (2^b - 1))``, 4-bit nibble packing (even
dimension in the high nibble, odd D zero-padded), and the same decode.  Codes and
reconstructions are bit-identical to numpy's, including numpy's dtype rules (f32 inputs
are quantized in f32, f64 inputs in f64; decode returns the dtype of min/max) and its
wrap-around cast of out-of-range values.  The element-wise work runs in
``mivq_sq_encode_*`` / ``mivq_sq_decode_*``.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _arrays, _native
from .base_quantizer import BaseQuantizer


class ScalarQuantizer(BaseQuantizer):
    def __init__(self, num_bits: int = 8):
        if num_bits not in [4, 8, 16]:
            raise ValueError(f"num_bits must be 4, 8, or 16, got {num_bits}")
        self.num_bits = num_bits
        self.num_levels = 2 ** num_bits
        self.min = None
        self.max = None
        if num_bits <= 8:
            self.dtype = np.uint8
            self.bytes_per_dim = 1
        else:
            self.dtype = np.uint16
            self.bytes_per_dim = 2
        self._dev = None  # (lo, den) device tensors in the fit dtype

    def fit(self, X):
        if _arrays.is_tensor(X):
            self.min = _arrays.to_host(X.amin(dim=0))
            self.max = _arrays.to_host(X.amax(dim=0))
        else:
            X = np.asarray(X)
            dt = X.dtype if X.dtype in (np.float32, np.float64) else np.result_type(X.dtype, np.float32)
            Xd = _arrays.to_device(X, torch.float64 if dt == np.float64 else torch.float32)
            self.min = _arrays.to_host(Xd.amin(dim=0))
            self.max = _arrays.to_host(Xd.amax(dim=0))
        self._dev = None

    def _params(self, dtype):
        """lo / den on the device; den = max - min + 1e-8 evaluated exactly as numpy does."""
        if self._dev is None or self._dev[0].dtype != dtype:
            np_dt = np.float64 if dtype == torch.float64 else np.float32
            mn = np.asarray(self.min)
            den = ((np.asarray(self.max) - mn) + 1e-8).astype(np_dt)  # in the fit dtype, then widened
            lo = mn.astype(np_dt)
            dev = _arrays.device()
            self._dev = (torch.from_numpy(np.ascontiguousarray(lo)).to(dev),
                         torch.from_numpy(np.ascontiguousarray(den.astype(np_dt))).to(dev))
        return self._dev

    def _work_dtype(self, x_dtype) -> torch.dtype:
        if isinstance(x_dtype, torch.dtype):
            x_dtype = torch.empty((), dtype=x_dtype).numpy().dtype
        rt = np.result_type(x_dtype, np.asarray(self.min).dtype)
        return torch.float64 if rt == np.float64 else torch.float32

    def compress(self, X):
        if self.min is None:
            raise RuntimeError("ScalarQuantizer must be fitted before compress().")
        if _arrays.is_tensor(X):
            wd = self._work_dtype(X.dtype)
            lo, den = self._params(wd)
            return _native.sq_encode(_arrays.to_device(X, wd), lo, den, self.num_bits)
        X = np.asarray(X)
        wd = self._work_dtype(X.dtype)
        lo, den = self._params(wd)
        n, d = X.shape
        width = (d + 1) // 2 if self.num_bits == 4 else d
        out = np.empty((n, width), dtype=self.dtype)
        esz = 8 if wd == torch.float64 else 4
        for s, e in _arrays.row_chunks(n, d * esz):
            codes = _native.sq_encode(_arrays.to_device(X[s:e], wd), lo, den, self.num_bits)
            h = _arrays.to_host(codes)
            out[s:e] = h.view(np.uint16) if self.num_bits == 16 else h
        return out

    def decompress(self, codes):
        if self.min is None:
            raise RuntimeError("ScalarQuantizer must be fitted before decompress().")
        md = torch.float64 if np.asarray(self.min).dtype == np.float64 else torch.float32
        lo, den = self._params(md)
        d = len(self.min)
        if _arrays.is_tensor(codes):
            return _native.sq_decode(codes.contiguous(), d, lo, den, self.num_bits)
        codes = np.ascontiguousarray(codes)
        if self.num_bits == 16:
            ct = torch.from_numpy(codes.astype(np.uint16).view(np.int16))
        else:
            ct = torch.from_numpy(codes.astype(np.uint8))
        n = codes.shape[0]
        out = np.empty((n, d), dtype=np.float64 if md == torch.float64 else np.float32)
        for s, e in _arrays.row_chunks(n, d * 8):
            rec = _native.sq_decode(ct[s:e].to(_arrays.device()).contiguous(), d, lo, den, self.num_bits)
            out[s:e] = _arrays.to_host(rec)
        return out

    def get_compression_ratio(self, X):
        original = X.shape[1] * 4
        if self.num_bits == 4:
            compressed = (X.shape[1] + 1) // 2
        else:
            compressed = X.shape[1] * self.bytes_per_dim
        return original / compressed
