"""RaBitQIndex — RaBitQ codes searched with the RaBitQ distance estimator, on the MI355X.

Drop-in for the reference's ``RaBitQIndex`` (/root/reference/src/haag_vq/methods/search/
rabitq_index.py:14-125), which wraps ``faiss.IndexRaBitQ(D, metric)`` with ``.qb = qb``:
train computes the center (mean of the training rows), add stores 1-bit codes of x - center
with the two per-vector factors, and search ranks every code by the RaBitQ estimator with
the query residual quantised to ``qb`` bits.  Here the codes are ``mivq_rabitq_encode``
rows (the RaBitQuantizer layout) and the search is ``mivq_rabitq_search`` (int8 MFMA over
the sign bits, estimator epilogue, tiled top-k).  faiss is absent, so the estimator's fp32
arithmetic is the restatement in oracle/mivq_oracle.c (parity unpinned vs faiss); the
center is the fp64 mean of the rows rounded to fp32.

Search returns ``(ids uint32, dists float32)``: squared-L2 estimates ascending, or
inner-product estimates descending (metric ``'ip'``).  ``save`` / ``load`` write an ``.npz``
of plain arrays (faiss' own index file format is not reproduced).
"""

from __future__ import annotations

from pathlib import Path
from typing import Literal, Optional, Tuple

import numpy as np
import torch

from ... import _arrays, _native
from ..base_search_index import BaseSearchIndex

_METRIC = {"l2": _native.METRIC_L2, "ip": _native.METRIC_INNER_PRODUCT}


class RaBitQIndex(BaseSearchIndex):
    """RaBitQ quantizer with native distance-estimator search (``qb`` query bits, 0..8)."""

    def __init__(self, qb: int = 4) -> None:
        self._qb = int(qb)
        if not 0 <= self._qb <= 8:
            raise ValueError(f"qb must be in [0, 8], got {qb}")
        self._codes: Optional[torch.Tensor] = None
        self._center: Optional[torch.Tensor] = None
        self._D: int = 0
        self._metric: Literal["l2", "ip"] = "l2"

    @property
    def ntotal(self) -> int:
        return 0 if self._codes is None else int(self._codes.shape[0])

    @property
    def code_size(self) -> int:
        return _native.rabitq_code_size(self._D)

    def fit(self, X, metric: Literal["l2", "ip"] = "l2") -> None:
        if metric not in _METRIC:
            raise ValueError(f"metric must be 'l2' or 'ip', got {metric!r}")
        Xd = _arrays.to_device(X, torch.float32)
        self._D = int(Xd.shape[1])
        self._metric = metric
        n = int(Xd.shape[0])
        center = Xd.double().sum(0) / max(n, 1) if n else torch.zeros(self._D, dtype=torch.float64, device=Xd.device)
        self._center = center.float().contiguous()
        self._codes = _native.rabitq_encode(Xd, self._center, _METRIC[metric])

    def _require_fit(self) -> torch.Tensor:
        if self._codes is None:
            raise RuntimeError("RaBitQIndex must be fit() before use.")
        return self._codes

    def search(self, Q, k: int) -> np.ndarray:
        ids, _ = self.search_with_scores(Q, k)
        return ids

    def search_device(self, Q, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Device-resident search: (dists f32 (nq, k), ids int32 (nq, k) holding uint32 ids)."""
        codes = self._require_fit()
        Qd = _arrays.to_device(Q, torch.float32)
        mt = _METRIC[self._metric]
        outs_d, outs_i = [], []
        for s in range(0, Qd.shape[0], 60000):  # query chunks (grid y of the generic kernel)
            d, i = _native.rabitq_search(codes, self._D, self._center, Qd[s:s + 60000].contiguous(), self._qb, mt, k)
            outs_d.append(-d if mt == _native.METRIC_INNER_PRODUCT else d)
            outs_i.append(i)
        return torch.cat(outs_d), torch.cat(outs_i)

    def search_with_scores(self, Q, k: int) -> Tuple[np.ndarray, np.ndarray]:
        self._require_fit()
        nq = int(Q.shape[0])
        k = min(int(k), self.ntotal)
        if k <= 0:
            return np.empty((nq, 0), dtype=np.uint32), np.empty((nq, 0), dtype=np.float32)
        d, i = self.search_device(Q, k)
        return _arrays.to_host(i).view(np.uint32), _arrays.to_host(d)

    def memory_footprint(self) -> int:
        if self._codes is None:
            return 0
        return self.ntotal * self.code_size

    def reconstruct_batch(self, ids) -> torch.Tensor:
        codes = self._require_fit()
        idx = torch.as_tensor(np.asarray(ids, dtype=np.int64), device=codes.device)
        return _native.rabitq_decode(codes[idx].contiguous(), self._D, self._center)

    def reconstruction_mse(self, X, sample_ids: Optional[np.ndarray] = None) -> Optional[float]:
        if self._codes is None:
            return None
        if sample_ids is None:
            sample_ids = np.arange(self.ntotal, dtype=np.int64)
        sample_ids = np.asarray(sample_ids, dtype=np.int64)
        X_hat = _arrays.to_host(self.reconstruct_batch(sample_ids)).astype(np.float32)
        X = np.asarray(X, dtype=np.float32)
        return float(np.mean((X[sample_ids] - X_hat) ** 2))

    def save(self, path: str | Path) -> None:
        if self._codes is None:
            raise RuntimeError("RaBitQIndex.save() called before fit()")
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        with open(path, "wb") as f:
            np.savez(f, codes=_arrays.to_host(self._codes), center=_arrays.to_host(self._center),
                     qb=np.array(self._qb), metric=np.array(self._metric), D=np.array(self._D))

    def load(self, path: str | Path) -> None:
        with np.load(Path(path), allow_pickle=False) as z:
            self._codes = _arrays.to_device(np.array(z["codes"]), torch.uint8)
            self._center = _arrays.to_device(np.array(z["center"]), torch.float32)
            self._qb = int(z["qb"])
            self._metric = str(z["metric"])
            self._D = int(z["D"])
