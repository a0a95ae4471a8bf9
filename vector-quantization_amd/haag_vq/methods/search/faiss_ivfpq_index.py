"""IVF-PQ index on the MI355X — drop-in for the reference's FaissIvfPqIndex.

Same constructor, methods and return types as
/root/reference/src/haag_vq/methods/search/faiss_ivfpq_index.py:14-107 (an external-baseline
wrapper of faiss.IndexIVFPQ): ``K`` coarse cells, ``m`` PQ subspaces of ``nbits`` bits,
``nprobe`` cells probed per query; ``fit`` trains the coarse quantizer and the residual PQ
on X and adds X; ``search`` returns uint32 ids, ``search_with_scores`` (ids, f32 distances)
with squared L2 ascending or inner product descending; ``memory_footprint`` uses the
reference's formula (:87-93); ``reconstruction_mse`` returns None as the reference does.

The engine is haag_vq.methods._ivf.IvfPq (coarse k-means, residual PQ, inverted lists, the
IVF-PQ scan kernel of libmivq).  ``save`` / ``load`` write an ``.npz`` of plain arrays
(loaded with allow_pickle=False) instead of a faiss index file.
"""

from __future__ import annotations

from pathlib import Path
from typing import Literal, Optional, Tuple

import numpy as np
import torch

from ... import _arrays, _native
from .._ivf import IvfLists, IvfPq
from ..base_search_index import BaseSearchIndex

_METRIC = {"l2": _native.METRIC_L2, "ip": _native.METRIC_INNER_PRODUCT}


class FaissIvfPqIndex(BaseSearchIndex):
    """IVF + residual PQ with ADC over the probed lists."""

    def __init__(self, K: int = 4096, m: int = 16, nbits: int = 8, nprobe: int = 200) -> None:
        self._K = K
        self._m = m
        self._nbits = nbits
        self._nprobe = nprobe
        self._index: Optional[IvfPq] = None
        self._metric: Literal["l2", "ip"] = "l2"
        self._N: int = 0
        self._D: int = 0

    @property
    def nprobe(self) -> int:
        return self._nprobe

    @nprobe.setter
    def nprobe(self, v: int) -> None:
        self._nprobe = int(v)

    def fit(self, X, metric: Literal["l2", "ip"] = "l2") -> None:
        if metric not in _METRIC:
            raise ValueError(f"unknown metric {metric!r}")
        Xd = _arrays.to_device(X)
        self._N, self._D = Xd.shape
        self._metric = metric
        self._index = IvfPq(self._D, self._K, self._m, self._nbits, _METRIC[metric])
        self._index.train(Xd)
        self._index.add(Xd)

    def _require(self) -> IvfPq:
        if self._index is None or self._index.lists is None:
            raise RuntimeError("index is not fitted; call fit() first")
        return self._index

    def _search(self, Q, k: int):
        idx = self._require()
        d, i = idx.search(_arrays.to_device(Q), k, self._nprobe)
        ids = _arrays.to_host(i).view(np.uint32)
        dists = _arrays.to_host(d)
        if self._metric == "ip":
            dists = -dists
        return ids, dists.astype(np.float32)

    def search(self, Q, k: int) -> np.ndarray:
        return self._search(Q, k)[0]

    def search_with_scores(self, Q, k: int) -> Tuple[np.ndarray, np.ndarray]:
        return self._search(Q, k)

    def memory_footprint(self) -> int:
        if self._index is None:
            return 0
        centroid_bytes = self._K * self._D * 4
        code_bytes = self._N * self._m
        codebook_bytes = self._D * (1 << self._nbits) * 4
        return centroid_bytes + code_bytes + codebook_bytes

    def reconstruction_mse(self, X, sample_ids: Optional[np.ndarray] = None) -> Optional[float]:
        return None  # as the reference (faiss_ivfpq_index.py:95-103)

    def save(self, path: str | Path) -> None:
        idx = self._require()
        L = idx.lists
        arrs = dict(
            meta=np.array([self._K, self._m, self._nbits, self._nprobe, self._N, self._D, _METRIC[self._metric]],
                          np.int64),
            coarse=_arrays.to_host(idx.coarse), pq=_arrays.to_host(idx.pq), offsets=_arrays.to_host(L.offsets),
            codes=_arrays.to_host(L.codes), ids=_arrays.to_host(L.ids),
        )
        if L.tau is not None:
            arrs["tau"] = _arrays.to_host(L.tau)
        with open(path, "wb") as f:
            np.savez(f, **arrs)

    def load(self, path: str | Path) -> None:
        with np.load(path, allow_pickle=False) as z:
            K, m, nbits, _nprobe, N, D, mt = (int(v) for v in z["meta"])
            self._K, self._m, self._nbits, self._N, self._D = K, m, nbits, N, D
            self._metric = "l2" if mt == _native.METRIC_L2 else "ip"
            idx = IvfPq(D, K, m, nbits, mt)
            dev = _arrays.device()
            idx.coarse = torch.from_numpy(z["coarse"]).to(dev)
            idx.pq = torch.from_numpy(z["pq"]).to(dev)
            idx.prep = _native.pq_prepare(idx.pq, nbits)
            idx.lists = IvfLists(offsets=torch.from_numpy(z["offsets"]).to(dev),
                                 codes=torch.from_numpy(z["codes"]).to(dev),
                                 ids=torch.from_numpy(z["ids"]).to(dev),
                                 tau=torch.from_numpy(z["tau"]).to(dev) if "tau" in z.files else None)
            idx.ntotal = N
        self._index = idx
