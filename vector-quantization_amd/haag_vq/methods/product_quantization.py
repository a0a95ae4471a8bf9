"""Product quantization on the MI355X.

Drop-in for the reference's ``ProductQuantizer``
(/root/reference/src/haag_vq/methods/product_quantization.py:9-99): same constructor
(``M``, ``B``, deprecated ``num_chunks`` / ``num_clusters`` aliases), same attributes
(``M``, ``B``, ``num_chunks``, ``num_clusters``, ``codebooks`` as a list of (ksub, dsub)
arrays, ``chunk_dim``, ``pq``), same errors, same code layout (faiss' PQ bit stream:
``code_size = ceil(M*B/8)`` bytes per vector).  ``compress`` / ``decompress`` run the HIP
kernels of libmivq.so (``mivq_pq_encode`` / ``mivq_pq_decode``); ``fit`` trains on the
GPU (``_kmeans.train_pq``).  numpy in -> numpy out; device tensors stay on the device.
"""

from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from .. import _arrays, _native
from ._kmeans import train_pq
from .base_quantizer import BaseQuantizer


class PQHandle:
    """Stands where the reference keeps its ``faiss.ProductQuantizer`` (``model.pq``).

    Exposes the attributes callers read (``d``, ``M``, ``nbits``, ``ksub``, ``dsub``,
    ``code_size``, ``centroids`` as the flat f32 vector) and faiss-style
    ``compute_codes`` / ``decode`` that run on the device.
    """

    def __init__(self, owner: "ProductQuantizer") -> None:
        self._owner = owner

    @property
    def d(self) -> int:
        return self._owner._C.shape[0] * self._owner._C.shape[2]

    @property
    def M(self) -> int:
        return self._owner.M

    @property
    def nbits(self) -> int:
        return self._owner.B

    @property
    def ksub(self) -> int:
        return 1 << self._owner.B

    @property
    def dsub(self) -> int:
        return int(self._owner.chunk_dim)

    @property
    def code_size(self) -> int:
        return _native.pq_code_size(self._owner.M, self._owner.B)

    @property
    def centroids(self) -> np.ndarray:
        return _arrays.to_host(self._owner._C).reshape(-1)

    def compute_codes(self, x):
        return self._owner.compress(x)

    def decode(self, codes):
        return self._owner.decompress(codes)


class ProductQuantizer(BaseQuantizer):
    def __init__(
        self,
        M: Optional[int] = None,
        B: int = 8,
        *,
        num_chunks: Optional[int] = None,
        num_clusters: Optional[int] = None,
    ):
        """Product quantization with M sub-quantizers of 2**B centroids each.

        Args mirror product_quantization.py:10-27 (``num_chunks`` / ``num_clusters`` are
        deprecated aliases of ``M`` / ``2**B``).
        """
        if M is None and num_chunks is not None:
            M = int(num_chunks)
        if num_chunks is not None and M is not None and int(num_chunks) != int(M):
            raise ValueError("Conflicting values for M and num_chunks")
        if num_clusters is not None:
            if num_clusters <= 0:
                raise ValueError("num_clusters must be positive")
            log2c = int(round(np.log2(num_clusters)))
            if 2 ** log2c != int(num_clusters):
                raise ValueError("num_clusters must be a power of two")
            B = log2c
        if M is None:
            M = 8
        self.M: int = int(M)
        self.B: int = int(B)
        if not 1 <= self.B <= 8:
            raise ValueError(f"B={self.B}: the MI355X build supports 1..8 bits per sub-code")
        self.num_chunks: int = self.M
        self.num_clusters: int = 2 ** self.B
        self.codebooks: List[np.ndarray] = []
        self.chunk_dim: Optional[int] = None
        self.pq: Optional[PQHandle] = None
        self._C: Optional[torch.Tensor] = None     # (M, ksub, dsub) f32, device
        self._prep: Optional[torch.Tensor] = None  # derived codebook data (mivq_pq_prepare)
        self.niter = 25
        self.seed = 1234

    # ------------------------------------------------------------------ state
    def set_codebooks(self, centroids) -> None:
        """Install (M, ksub, dsub) centroids (e.g. loaded from disk) and prepare them."""
        C = _arrays.to_device(centroids, torch.float32)
        if C.dim() != 3 or C.shape[0] != self.M or C.shape[1] != (1 << self.B):
            raise ValueError(f"centroids must be ({self.M}, {1 << self.B}, dsub), got {tuple(C.shape)}")
        self._C = C.contiguous()
        self.chunk_dim = int(C.shape[2])
        self._prep = _native.pq_prepare(self._C, self.B)
        host = _arrays.to_host(self._C)
        self.codebooks = [np.array(host[m], copy=True) for m in range(self.M)]
        self.pq = PQHandle(self)

    @property
    def centroids_device(self) -> torch.Tensor:
        self._require_fitted("compress")
        return self._C

    def _require_fitted(self, what: str) -> None:
        if self._C is None:
            raise RuntimeError(f"ProductQuantizer must be fitted before {what}(). Call fit() first.")

    # ------------------------------------------------------------------ API
    def fit(self, X) -> None:
        Xd = _arrays.to_device(X, torch.float32)
        N, D = Xd.shape
        if D % self.M != 0:
            raise AssertionError("D must be divisible by M (number of subquantizers)")
        self.chunk_dim = D // self.M
        C = train_pq(Xd, self.M, self.B, niter=self.niter, seed=self.seed)
        self.set_codebooks(C)

    def compress(self, X):
        self._require_fitted("compress")
        if _arrays.is_tensor(X):
            return _native.pq_encode(_arrays.to_device(X), self._C, self._prep, self.B)
        X = np.asarray(X, dtype=np.float32)
        if X.ndim != 2 or X.shape[1] != self.M * self.chunk_dim:
            raise ValueError(f"compress: expected (n, {self.M * self.chunk_dim}) input, got {X.shape}")
        n = X.shape[0]
        out = np.empty((n, _native.pq_code_size(self.M, self.B)), dtype=np.uint8)
        for s, e in _arrays.row_chunks(n, X.shape[1] * 4):
            codes = _native.pq_encode(_arrays.to_device(X[s:e]), self._C, self._prep, self.B)
            out[s:e] = _arrays.to_host(codes)
        return out

    def decompress(self, codes):
        self._require_fitted("decompress")
        if _arrays.is_tensor(codes):
            return _native.pq_decode(_arrays.to_device(codes, torch.uint8), self._C, self.B)
        codes = np.asarray(codes)
        if codes.ndim == 1:
            codes = codes.reshape(1, -1)
        n = codes.shape[0]
        D = self.M * self.chunk_dim
        out = np.empty((n, D), dtype=np.float32)
        for s, e in _arrays.row_chunks(n, D * 4):
            rec = _native.pq_decode(_arrays.to_device(codes[s:e], torch.uint8), self._C, self.B)
            out[s:e] = _arrays.to_host(rec)
        return out

    def get_compression_ratio(self, X) -> float:
        """Original bytes (float32) over code bytes — product_quantization.py:88-99."""
        D = int(X.shape[1])
        return float(D * 4 / _native.pq_code_size(self.M, self.B))
