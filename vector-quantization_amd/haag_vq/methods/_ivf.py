"""Inverted-file (IVF) machinery on the MI355X: coarse k-means, list assignment, IVF-PQ.

Replaces what faiss ``IndexIVFPQ`` does inside FaissIvfPqIndex
(/root/reference/src/haag_vq/methods/search/faiss_ivfpq_index.py:46-76) and the IVF build
of benchmarks/ivf_benchmark.py:170-204:

* ``train_coarse``  the coarse quantizer's k-means (faiss' IVF clustering shape: a random
  sample of at most 256 points per centroid, seed 1234, centroids initialised from the
  sample, 10 Lloyd iterations, empty clusters re-seeded by splitting).  Assignment is the
  exact pairwise-distance kernel + a per-row argmin; the update is the ascending-row
  centroid sum over a stable bucket sort, so a fit is bit-reproducible.
* ``IvfPq``  residual product quantization (faiss' ``by_residual``): PQ codebooks trained on
  residuals x - coarse[list(x)], codes from the bit-exact PQ encode of the residuals, lists
  in bucket order, and the per-vector L2 term tau_i that turns faiss' per-list
  precomputed table into one number per code, so a query needs only its own M x ksub LUT:
      ||q - c_l - r_i||^2 = ||q - c_l||^2 + tau_i - 2 q.r_i,  tau_i = ||r_i||^2 + 2 c_l.r_i.
  IP (IndexFlatIP quantizer): score = q.c_l + q.r_i, ranked as its negation.

faiss itself is absent here, so coarse centroids, codebooks and results are not claimed to
equal faiss'; the arithmetic is the canonical one of include/mivq.h and oracle/.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch

from .. import _native
from ._kmeans import EPS, train_pq

_MAT_BYTES = 1 << 30  # per-chunk (rows x K) distance matrix budget


def _rows_per_chunk(K: int) -> int:
    return max(1, _MAT_BYTES // (4 * max(1, K)))


def assign(X: torch.Tensor, C: torch.Tensor, metric: int = _native.METRIC_L2) -> Tuple[torch.Tensor, torch.Tensor]:
    """Nearest coarse centroid of every row: (dist f32 (n,), list int32 (n,))."""
    n = X.shape[0]
    K = C.shape[0]
    dd = torch.empty(n, dtype=torch.float32, device=X.device)
    ll = torch.empty(n, dtype=torch.int32, device=X.device)
    step = _rows_per_chunk(K)
    buf = None
    for s in range(0, n, step):
        e = min(n, s + step)
        if buf is None or buf.shape[0] != e - s:
            buf = torch.empty((e - s, K), dtype=torch.float32, device=X.device)
        _native.pairwise_distances(X[s:e], C, metric, out=buf)
        d1, i1 = _native.topk_rows(buf, 1)
        dd[s:e] = d1[:, 0]
        ll[s:e] = i1[:, 0]
    return dd, ll


def _split_empty(C: np.ndarray, cnt: np.ndarray, rng: np.random.Generator, n: int) -> int:
    """faiss-style split of empty clusters of a (K, d) codebook, in place."""
    K, d = C.shape
    cnt = cnt.astype(np.float64)
    nsplit = 0
    sign = np.where(np.arange(d) % 2 == 0, 1.0, -1.0).astype(np.float32)
    for ci in range(K):
        if cnt[ci] != 0:
            continue
        cj = 0
        denom = max(1.0, float(n - K))
        for _ in range(64 * K):
            if rng.random() < (cnt[cj] - 1.0) / denom:
                break
            cj = (cj + 1) % K
        else:
            cj = int(np.argmax(cnt))
        C[ci] = C[cj]
        C[ci] *= (1.0 + EPS * sign).astype(np.float32)
        C[cj] *= (1.0 - EPS * sign).astype(np.float32)
        cnt[ci] = np.floor(cnt[cj] / 2)
        cnt[cj] -= cnt[ci]
        nsplit += 1
    return nsplit


def train_coarse(X: torch.Tensor, K: int, niter: int = 10, seed: int = 1234, max_points_per_centroid: int = 256,
                 metric: int = _native.METRIC_L2) -> torch.Tensor:
    """(K, d) f32 coarse centroids by Lloyd iterations on a sample of device rows X."""
    n, d = X.shape
    if n < K:
        raise RuntimeError(f"Number of training points ({n}) should be at least as large as number of clusters ({K})")
    rng = np.random.default_rng(seed)
    max_n = max_points_per_centroid * K
    if n > max_n:
        sel = np.sort(rng.permutation(n)[:max_n])
        Xt = X[torch.from_numpy(sel).to(X.device)].contiguous()
    else:
        Xt = X.contiguous()
    nt = Xt.shape[0]
    pick = np.sort(rng.permutation(nt)[:K])
    C = Xt[torch.from_numpy(pick).to(X.device)].contiguous().clone()
    counts = torch.empty(K, dtype=torch.int32, device=X.device)
    for _ in range(niter):
        _, a = assign(Xt, C, metric)
        offsets, order = _native.bucket_sort(a, K)
        _native.centroid_update(Xt, offsets, order, C, counts)
        cnt = counts.cpu().numpy()
        if (cnt == 0).any():
            Ch = C.cpu().numpy()
            _split_empty(Ch, cnt, rng, nt)
            C = torch.from_numpy(Ch).to(X.device).contiguous()
    return C


@dataclass
class IvfLists:
    """Inverted lists in bucket order (device tensors)."""
    offsets: torch.Tensor     # (K+1,) int64
    codes: torch.Tensor       # (N, M) uint8, one byte per sub-code
    ids: torch.Tensor         # (N,) int32 holding uint32 ids
    tau: Optional[torch.Tensor]  # (N,) f32, L2 only


class IvfPq:
    """IVF with residual PQ (device-resident); the engine behind FaissIvfPqIndex."""

    def __init__(self, d: int, K: int, M: int, nbits: int = 8, metric: int = _native.METRIC_L2) -> None:
        if d % M != 0:
            raise AssertionError("D must be divisible by M (number of subquantizers)")
        self.d, self.K, self.M, self.nbits, self.metric = d, K, M, nbits, metric
        self.coarse: Optional[torch.Tensor] = None
        self.pq: Optional[torch.Tensor] = None    # (M, ksub, dsub)
        self.prep: Optional[torch.Tensor] = None
        self.lists: Optional[IvfLists] = None
        self.ntotal = 0

    # --------------------------------------------------------------- train / add
    def train(self, X: torch.Tensor, coarse_iters: int = 10, pq_iters: int = 25, seed: int = 1234) -> None:
        self.coarse = train_coarse(X, self.K, niter=coarse_iters, seed=seed, metric=self.metric)
        ksub = 1 << self.nbits
        rng = np.random.default_rng(seed + 1)
        n = X.shape[0]
        cap = 256 * ksub
        Xs = X if n <= cap else X[torch.from_numpy(np.sort(rng.permutation(n)[:cap])).to(X.device)].contiguous()
        _, a = assign(Xs, self.coarse, self.metric)
        R = _native.ivf_residuals(Xs, self.coarse, a)
        self.pq = train_pq(R, self.M, self.nbits, niter=pq_iters, seed=seed)
        self.prep = _native.pq_prepare(self.pq, self.nbits)

    def _encode(self, X: torch.Tensor):
        n = X.shape[0]
        a = torch.empty(n, dtype=torch.int32, device=X.device)
        codes = torch.empty((n, self.M), dtype=torch.uint8, device=X.device)
        tau = torch.empty(n, dtype=torch.float32, device=X.device) if self.metric == _native.METRIC_L2 else None
        step = max(1, min(_rows_per_chunk(self.K), (1 << 30) // (4 * self.d)))
        for s in range(0, n, step):
            e = min(n, s + step)
            _, a[s:e] = assign(X[s:e], self.coarse, self.metric)
            R = _native.ivf_residuals(X[s:e], self.coarse, a[s:e])
            c = _native.pq_encode(R, self.pq, self.prep, self.nbits)
            u8 = c if self.nbits == 8 else _native.pq_unpack(c, self.M, self.nbits)
            codes[s:e] = u8
            if tau is not None:
                tau[s:e] = _native.ivfpq_terms(u8, self.pq, self.prep, self.coarse, a[s:e], self.nbits)
        return a, codes, tau

    def add(self, X: torch.Tensor) -> None:
        """Append rows (ids continue from ntotal); lists are rebuilt in bucket order."""
        a, codes, tau = self._encode(X)
        ids = torch.arange(self.ntotal, self.ntotal + X.shape[0], dtype=torch.int64, device=X.device).to(torch.int32)
        if self.lists is not None and self.ntotal > 0:
            old = self.lists
            # recover the row-order arrays of the existing lists from their bucket order
            a_old = torch.repeat_interleave(torch.arange(self.K, dtype=torch.int32, device=X.device),
                                            (old.offsets[1:] - old.offsets[:-1]))
            a = torch.cat([a_old, a])
            codes = torch.cat([old.codes, codes])
            ids = torch.cat([old.ids, ids])
            if tau is not None:
                tau = torch.cat([old.tau, tau])
        offsets, order = _native.bucket_sort(a.contiguous(), self.K)
        self.lists = IvfLists(
            offsets=offsets,
            codes=_native.gather_rows(codes.contiguous(), order) if self.M % 4 == 0 else codes[order.long()].contiguous(),
            ids=_native.gather_rows(ids.contiguous(), order),
            tau=None if tau is None else _native.gather_rows(tau.contiguous(), order),
        )
        self.ntotal += X.shape[0]

    # --------------------------------------------------------------- search
    def search(self, Q: torch.Tensor, k: int, nprobe: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """(dists f32 (nq, k), ids int32 (nq, k)); L2 ascending, IP as negated scores."""
        nprobe = max(1, min(int(nprobe), self.K))
        if nprobe > 256:
            raise ValueError(f"nprobe={nprobe}: the probe selection (mivq_topk_rows) supports at most 256 lists")
        pd, pl = _native.topk_rows(_native.pairwise_distances(Q, self.coarse, self.metric), nprobe)
        lut = _native.adc_lut(Q, self.pq, self.nbits, _native.METRIC_INNER_PRODUCT)
        L = self.lists
        return _native.ivfpq_search(lut, pd, pl, L.offsets, L.codes, L.ids, L.tau, self.metric, k, self.nbits)
