"""Optimized product quantization (OPQ) on the MI355X.

Drop-in for the reference's ``OptimizedProductQuantizer``
(/root/reference/src/haag_vq/methods/optimized_product_quantization.py:7-46), which wraps
``faiss.OPQMatrix(D, M, D)`` + ``faiss.ProductQuantizer``:

* fit: learn an orthonormal rotation A by the OPQ alternating optimisation faiss'
  OPQMatrix documents (random orthonormal init from seed 1234, ``niter`` rounds of
  {rotate the <= 65536-row training sample, train PQ (40 k-means iterations the first
  round, 4 warm-started ones after), encode+decode, orthogonal-Procrustes update of A}),
  then train a fresh PQ on the rotated data (:26-28).
* compress = PQ encode of x . A^T (:31); decompress = PQ decode . A (:34).

Hot path on device: the rotation is ``mivq_opq_rotate_prepared`` (hand-written split-f16
MFMA GEMM with fp32 accuracy; the f16 hi / lo image of A is prepared once per matrix and
direction), encode / decode are the PQ kernels.  ``mivq_opq_rotate`` (plain fp32 MFMA, no
preparation) serves dimensions that are not multiples of 8.  The Procrustes step of training
runs on repo kernels too (round 4): the fp64 Gram matrix X^T Yhat on ``mivq_opq_gram`` and the
polar factor of it by a Newton-Schulz iteration on the fp64 MFMA GEMM (``polar_factor``), with
torch's SVD only as the fallback for a matrix the iteration cannot orthogonalise.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _arrays, _native
from ._kmeans import train_pq
from .base_quantizer import BaseQuantizer
from .product_quantization import ProductQuantizer


def rotate(x: torch.Tensor, A: torch.Tensor, transpose: bool = False, prep=None,
           out: torch.Tensor | None = None) -> torch.Tensor:
    """x . A^T (transpose False) or x . A on the device: the prepared split-f16 GEMM when
    A's image is available (d % 8 == 0), else the plain fp32 MFMA kernel."""
    if prep is None:
        prep = _native.opq_prepare(A, transpose)
    if prep is None:
        return _native.opq_rotate(x, A, transpose, out=out)
    return _native.opq_rotate_prepared(x, prep, out=out)


class OPQHandle:
    """Stands where the reference keeps ``faiss.OPQMatrix`` (``model.opq``)."""

    def __init__(self, A: torch.Tensor) -> None:
        self.A_device = A
        self.d_in = self.d_out = int(A.shape[0])
        self.is_orthonormal = True
        self._prep = {}

    def prep(self, transpose: bool):
        """The prepared image of A^T (apply) or A (reverse), built on first use."""
        if transpose not in self._prep:
            self._prep[transpose] = _native.opq_prepare(self.A_device, transpose)
        return self._prep[transpose]

    def rotate(self, x: torch.Tensor, transpose: bool, out: torch.Tensor | None = None) -> torch.Tensor:
        return rotate(x, self.A_device, transpose, prep=self.prep(transpose), out=out)

    @property
    def A(self) -> np.ndarray:
        return _arrays.to_host(self.A_device).reshape(-1)

    def _run(self, x, transpose: bool):
        if _arrays.is_tensor(x):
            return self.rotate(_arrays.to_device(x), transpose)
        x = np.asarray(x, dtype=np.float32)
        out = np.empty_like(x)
        for s, e in _arrays.row_chunks(x.shape[0], x.shape[1] * 8):
            out[s:e] = _arrays.to_host(self.rotate(_arrays.to_device(x[s:e]), transpose))
        return out

    def apply(self, x):
        """y = x . A^T (faiss LinearTransform::apply)."""
        return self._run(x, False)

    def reverse_transform(self, y):
        """x = y . A (inverse of an orthonormal A)."""
        return self._run(y, True)


def _mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a . b for square fp64 device matrices on the library's fp64 MFMA GEMM."""
    return _native.extrabitq_rotate(a.contiguous(), b.contiguous(), False)


def polar_factor(G: torch.Tensor, tol: float = 1e-13, max_iter: int = 60, info: dict | None = None) -> torch.Tensor:
    """The orthogonal polar factor Q = U V^T of a square fp64 matrix G = U S V^T (what
    faiss OPQMatrix::train takes from its SVD), by the Newton-Schulz iteration
    Q <- Q (3 I - Q^T Q) / 2 on the fp64 MFMA GEMM (erq_rotate_kernel) instead of rocsolver's
    SVD.  Start: G divided by an UPPER bound of its largest singular value,
    min(||G||_F, sqrt(||G^T G||_inf)), so every scaled singular value lies in (0, 1] and the
    iteration takes each of them to +1 (a start value above sqrt(3) goes to -1 or diverges, and
    an estimate from below -- e.g. a power iteration whose start vector misses the top singular
    vector -- cannot rule that out).  It doubles the digits once every singular value is near 1,
    and stops at ||Q^T Q - I||_F < tol sqrt(d) or once that error stalls at the fp64 rounding
    floor of the GEMMs.  A G the iteration cannot orthogonalise (rank deficient, or not
    converged within max_iter, or singular values below ~1e-6 of the top, whose growth the
    trace test below cannot see in fp64) falls back to the SVD; a
    rank-deficient G is recognised by its error stalling above 1e-8 (the zero singular values
    stay at zero, ||Q^T Q - I|| levels off at sqrt(#zeros)) for 4 steps while trace(Q^T Q) =
    sum sigma^2 stays put, not after max_iter.  Small but non-zero singular values (a tail of
    low-variance directions, e.g. 1e-3 of the top) also hold the error near sqrt(#small) for a
    while, but they grow by 1.5x per step, so the trace moves and the iteration goes on
    (the error test alone sent such G to the SVD).
    ``info`` (optional dict) receives {"path": "newton-schulz" | "svd", "iters": steps}."""
    d = G.shape[0]
    I = torch.eye(d, dtype=torch.float64, device=G.device)
    GtG = _mm(G.T, G)
    bound = min(float(G.norm()), float(GtG.abs().sum(dim=1).max()) ** 0.5)
    if bound > 0.0 and bound < float("inf"):
        Q = G / bound
        prev, prev_tr, stall = float("inf"), float("nan"), 0
        for it in range(max_iter):
            T = _mm(Q.T, Q)
            err = float((T - I).norm())
            tr = float(T.diagonal().sum())
            if err < tol * d ** 0.5 or (err < 1e-8 and err > 0.25 * prev):
                if info is not None:
                    info.update(path="newton-schulz", iters=it)
                return Q  # converged (quadratic phase stalled: the rounding floor)
            if not err < 1e3:  # non-finite
                break
            # levelled off above 1e-8 with sum sigma^2 not moving: zero singular values
            stall = stall + 1 if err >= 0.999 * prev and abs(tr - prev_tr) <= 1e-12 * d else 0
            if stall >= 4:
                break
            prev, prev_tr = err, tr
            Q = 1.5 * Q - 0.5 * _mm(Q, T)
    if info is not None:
        info.update(path="svd", iters=it + 1 if bound > 0.0 and bound < float("inf") else 0)
    U, _, Vh = torch.linalg.svd(G)
    return U @ Vh


class OptimizedProductQuantizer(BaseQuantizer):
    def __init__(self, M: int, B: int = 8):
        """OPQ (Ge et al., TPAMI 2013).  M sub-quantizers of 2**B centroids."""
        self.M = M
        self.B = B
        self.opq: OPQHandle | None = None
        self.pq = None
        self._inner: ProductQuantizer | None = None
        # OPQMatrix training parameters (faiss defaults)
        self.niter = 50
        self.niter_pq = 4
        self.niter_pq_0 = 40
        self.max_train_points = 256 * 256
        self.seed = 1234

    def _train_rotation(self, X: torch.Tensor) -> torch.Tensor:
        n, d = X.shape
        rng = np.random.default_rng(self.seed)
        if n > self.max_train_points:
            sel = np.sort(rng.permutation(n)[: self.max_train_points])
            X = X[torch.from_numpy(sel).to(X.device)].contiguous()
        A = self.initial_rotation(d, X.device)
        C = None
        for it in range(self.niter):
            A, C, _, _ = self.train_step(X, A, C, it)
        return A

    def initial_rotation(self, d: int, device) -> torch.Tensor:
        """Random orthonormal start (QR of a seeded Gaussian matrix)."""
        Q, _ = np.linalg.qr(np.random.default_rng(self.seed).standard_normal((d, d)))
        return torch.from_numpy(Q.astype(np.float32)).to(device).contiguous()

    def train_step(self, X: torch.Tensor, A: torch.Tensor, C, it: int):
        """One round of the alternating optimisation: rotate, (re)train PQ on the rotated
        sample, encode + decode, orthogonal-Procrustes update.  Returns (A', C, Y, Yhat)."""
        Y = rotate(X, A, False)
        C = train_pq(Y, self.M, self.B, niter=self.niter_pq_0 if it == 0 else self.niter_pq,
                     seed=self.seed, max_points_per_centroid=1000, init=C)
        prep = _native.pq_prepare(C, self.B)
        Yhat = _native.pq_decode(_native.pq_encode(Y, C, prep, self.B), C, self.B)
        # orthogonal Procrustes: argmin_R ||X R^T - Yhat||  ->  R = V U^T = Q^T with
        # X^T Yhat = U S V^T and Q = U V^T its orthogonal polar factor
        G = _native.opq_gram(X, Yhat)
        return polar_factor(G).T.float().contiguous(), C, Y, Yhat

    def fit(self, X) -> None:
        Xd = _arrays.to_device(X, torch.float32)
        N, D = Xd.shape
        assert D % self.M == 0, "D must be divisible by M"
        A = self._train_rotation(Xd)
        self.opq = OPQHandle(A)
        inner = ProductQuantizer(M=self.M, B=self.B)
        inner.fit(self.opq.rotate(Xd, False))
        self._inner = inner
        self.pq = inner.pq

    def _require(self, what: str) -> None:
        if self._inner is None or self.opq is None:
            raise RuntimeError(f"OptimizedProductQuantizer must be fitted before {what}().")

    def compress(self, X):
        self._require("compress")
        if _arrays.is_tensor(X):
            return self._inner.compress(self.opq.apply(X))
        X = np.asarray(X, dtype=np.float32)
        out = np.empty((X.shape[0], _native.pq_code_size(self.M, self.B)), dtype=np.uint8)
        for s, e in _arrays.row_chunks(X.shape[0], X.shape[1] * 8):
            y = self.opq.rotate(_arrays.to_device(X[s:e]), False)
            out[s:e] = _arrays.to_host(self._inner.compress(y))
        return out

    def decompress(self, compressed):
        self._require("decompress")
        if _arrays.is_tensor(compressed):
            return self.opq.reverse_transform(self._inner.decompress(compressed))
        compressed = np.asarray(compressed)
        D = self.M * self._inner.chunk_dim
        out = np.empty((compressed.shape[0], D), dtype=np.float32)
        for s, e in _arrays.row_chunks(compressed.shape[0], D * 8):
            c = _arrays.to_device(compressed[s:e], torch.uint8)
            out[s:e] = _arrays.to_host(self.opq.reverse_transform(self._inner.decompress(c)))
        return out

    @property
    def inner(self) -> ProductQuantizer:
        self._require("inner")
        return self._inner

    def get_compression_ratio(self, X) -> float:
        """D*4 / ceil(M*B/8) — optimized_product_quantization.py:36-46."""
        D = int(X.shape[1])
        return float(D * 4 / int((self.M * self.B + 7) // 8))
