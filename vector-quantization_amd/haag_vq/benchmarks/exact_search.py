"""Chunked exact search for the quantizer study, on the MI355X.

Same functions as /root/reference/src/haag_vq/benchmarks/exact_search.py:20-122.  The
reference ranks q . (x_hat / ||x||) with faiss IndexFlatIP; here ``ScaledIPIndex`` keeps the
scaled reconstructions on the device and ranks them with ``mivq_flat_search`` (IP).
"""

from __future__ import annotations

from typing import Callable, Dict, Iterator, Tuple

import numpy as np
import torch

from haag_vq import _arrays, _native

ReconstructFn = Callable[[np.ndarray], np.ndarray]


def compute_exact_norms(X: np.ndarray, eps: float = 1e-12) -> np.ndarray:
    norms = np.linalg.norm(np.asarray(X, dtype=np.float32), axis=1)
    return np.maximum(norms, eps).astype(np.float32)


def _chunks(n: int, chunk: int) -> Iterator[np.ndarray]:
    for s in range(0, n, chunk):
        yield np.arange(s, min(s + chunk, n), dtype=np.uint32)


class ScaledIPIndex:
    """Device-resident flat inner-product index (stands in for faiss.IndexFlatIP)."""

    def __init__(self, d: int) -> None:
        self.d = d
        self._parts = []

    @property
    def ntotal(self) -> int:
        return sum(p.shape[0] for p in self._parts)

    def add(self, x) -> None:
        self._parts.append(_arrays.to_device(x))

    def search(self, Q, k: int) -> Tuple[np.ndarray, np.ndarray]:
        X = self._parts[0] if len(self._parts) == 1 else torch.cat(self._parts).contiguous()
        self._parts = [X]
        k = min(int(k), X.shape[0])
        d, i = _native.flat_search(_arrays.to_device(Q), X, k, _native.METRIC_INNER_PRODUCT)
        return _arrays.to_host(-d), _arrays.to_host(i).view(np.uint32).astype(np.int64)


def build_scaled_ip_index(reconstruct_fn: ReconstructFn, n: int, d: int, norms: np.ndarray,
                          chunk: int = 50_000) -> ScaledIPIndex:
    index = ScaledIPIndex(d)
    for ids in _chunks(n, chunk):
        x_hat = np.ascontiguousarray(reconstruct_fn(ids), dtype=np.float32)
        x_hat *= (1.0 / norms[ids])[:, None]
        index.add(x_hat)
    return index


def search_index(index, Q: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    scores, ids = index.search(np.ascontiguousarray(Q, dtype=np.float32), k)
    assert (ids >= 0).all()
    return scores.astype(np.float32), ids.astype(np.uint32)


def normalized_ground_truth(X: np.ndarray, Q: np.ndarray, k: int, norms: np.ndarray | None = None,
                            chunk: int = 50_000) -> np.ndarray:
    X = np.asarray(X, dtype=np.float32)
    if norms is None:
        norms = compute_exact_norms(X)
    index = build_scaled_ip_index(lambda ids: X[ids], X.shape[0], X.shape[1], norms, chunk=chunk)
    _, ids = search_index(index, Q, k=k)
    return ids


def recall_at_ks(retrieved_ids: np.ndarray, gt_ids: np.ndarray, ks: Tuple[int, ...] = (1, 10, 100)) -> Dict[int, float]:
    nq = retrieved_ids.shape[0]
    out: Dict[int, float] = {}
    for k in ks:
        kr = min(k, retrieved_ids.shape[1])
        kg = min(k, gt_ids.shape[1])
        denom = min(kr, kg)
        if denom == 0:
            out[k] = 0.0
            continue
        total = 0.0
        for i in range(nq):
            total += len(set(gt_ids[i, :kg].tolist()) & set(retrieved_ids[i, :kr].tolist())) / denom
        out[k] = total / nq if nq else 0.0
    return out


def reconstruction_mse(X: np.ndarray, reconstruct_fn: ReconstructFn, sample_ids: np.ndarray,
                       chunk: int = 50_000) -> float:
    X = np.asarray(X, dtype=np.float32)
    sample_ids = np.asarray(sample_ids, dtype=np.uint32)
    d = X.shape[1]
    sq, cnt = 0.0, 0
    for s in range(0, sample_ids.size, chunk):
        blk = sample_ids[s:s + chunk]
        diff = X[blk] - np.asarray(reconstruct_fn(blk), dtype=np.float32)
        sq += float(np.sum(diff * diff))
        cnt += blk.size * d
    return sq / cnt if cnt else 0.0
