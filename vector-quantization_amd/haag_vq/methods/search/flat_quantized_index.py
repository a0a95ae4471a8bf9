"""Flat (brute-force) search over quantized codes, on the MI355X.

``FlatQuantizedIndex`` keeps the interface of the reference's class
(/root/reference/src/haag_vq/methods/search/flat_quantized_index.py:17-154): fit compresses
the database, ``search_with_scores`` returns ``(ids uint32, dists float32)`` sorted best
first (squared L2 ascending, or inner product descending), ``memory_footprint`` is the code
bytes, ``save`` / ``load`` round-trip the index.  The reference decodes every code and runs
``scipy.cdist`` + ``argpartition``; here:

* PQ / OPQ codes are ranked by ADC — per-query lookup tables (``mivq_adc_lut``) summed over
  the codes (``mivq_adc_search``).  sum_m ||q_m - c_{m,code_m}||^2 equals ||q - x_hat||^2
  (OPQ: for the rotated query, which the orthonormal rotation preserves), so the ranking is
  the reference's up to fp32 rounding on near-ties, without materialising x_hat.
* other quantizers (SQ, RaBitQ, ...) are decoded on the device and searched exactly
  (``mivq_flat_search``).

Ties are broken by the smaller id.  Saved indices are ``.npz`` archives of plain arrays
(loaded with ``allow_pickle=False``).
"""

from __future__ import annotations

from pathlib import Path
from typing import Literal, Optional, Tuple

import numpy as np
import torch

from ... import _arrays, _native
from ..base_quantizer import BaseQuantizer
from ..base_search_index import BaseSearchIndex
from ..optimized_product_quantization import OptimizedProductQuantizer, OPQHandle
from ..product_quantization import ProductQuantizer
from ..rabit_quantization import RaBitQuantizer
from ..scalar_quantization import ScalarQuantizer

_METRIC = {"l2": _native.METRIC_L2, "ip": _native.METRIC_INNER_PRODUCT}


def search_codes(model: BaseQuantizer, codes, Q, k: int, metric: str = "l2",
                 id_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Top-k of queries Q against encoded database ``codes`` of ``model`` (device tensors).

    Returns (dists f32 (nq, k), ids int32 (nq, k) holding uint32 ids); IP distances are
    returned as inner products (descending).  ``id_offset`` is added to every id (the first
    global row of a database shard, parallel/sharded.py).
    """
    mt = _METRIC[metric]
    Qd = _arrays.to_device(Q)
    cd = codes if _arrays.is_tensor(codes) else torch.from_numpy(np.ascontiguousarray(codes))
    cd = cd.to(_arrays.device())
    if k > MAX_KERNEL_K:
        d, i = _search_large_k(model, cd, Qd, k, mt)
        if id_offset:
            # ids are uint32 bit patterns in int32: mask before adding, and keep the
            # 0xFFFFFFFF sentinel as it is
            g = ((i.to(torch.int64) & 0xFFFFFFFF) + id_offset) & 0xFFFFFFFF
            i = torch.where(i == -1, i, (g - (g >= 2 ** 31).to(torch.int64) * 2 ** 32).to(torch.int32))
        return d, i
    if isinstance(model, (ProductQuantizer, OptimizedProductQuantizer)):
        pq = model if isinstance(model, ProductQuantizer) else model.inner
        if isinstance(model, OptimizedProductQuantizer):
            Qd = model.opq.apply(Qd)
        cd = cd.to(torch.uint8).contiguous()
        u8 = cd if pq.B == 8 else _native.pq_unpack(cd, pq.M, pq.B)
        lut = _native.adc_lut(Qd, pq.centroids_device, pq.B, mt)
        d, i = _native.adc_search(lut, u8, k, pq.B, id_offset=id_offset)
    else:
        xh = model.decompress(cd)
        xh = _arrays.to_device(xh, torch.float32)
        d, i = _native.flat_search(Qd, xh, k, mt, id_offset=id_offset)
    if mt == _native.METRIC_INNER_PRODUCT:
        d = -d
    return d, i


MAX_KERNEL_K = 256  # the wave-resident top-k of the scan kernels


def _search_large_k(model, cd, Qd, k: int, mt: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """k > 256 (the reference's cdist + argpartition has no limit): decode once, exact
    (query, row) distances with mivq_pairwise_distances in query blocks, and a stable
    device sort, so ties keep the smaller id first."""
    xh = _arrays.to_device(model.decompress(cd), torch.float32)
    n = xh.shape[0]
    k = min(k, n)
    block = max(1, (1 << 28) // max(1, n))
    ds, is_ = [], []
    for s in range(0, Qd.shape[0], block):
        D = _native.pairwise_distances(Qd[s:s + block].contiguous(), xh, mt)
        v, i = torch.sort(D, dim=1, stable=True)
        ds.append(v[:, :k].contiguous())
        is_.append(i[:, :k].to(torch.int32).contiguous())
    d, i = torch.cat(ds), torch.cat(is_)
    if mt == _native.METRIC_INNER_PRODUCT:
        d = -d
    return d, i


def ids_to_numpy(i: torch.Tensor) -> np.ndarray:
    return _arrays.to_host(i).view(np.uint32)


def quantizer_state(q: BaseQuantizer) -> dict:
    """A fitted quantizer as plain numpy arrays (index files; the rank-0 -> all-ranks
    broadcast of parallel/sharded.py)."""
    if isinstance(q, ProductQuantizer):
        return dict(qtype=np.array("pq"), M=np.array(q.M), B=np.array(q.B), centroids=_arrays.to_host(q._C))
    if isinstance(q, OptimizedProductQuantizer):
        return dict(qtype=np.array("opq"), M=np.array(q.M), B=np.array(q.B), A=_arrays.to_host(q.opq.A_device),
                    centroids=_arrays.to_host(q.inner._C))
    if isinstance(q, ScalarQuantizer):
        return dict(qtype=np.array("sq"), num_bits=np.array(q.num_bits), min=np.asarray(q.min), max=np.asarray(q.max))
    if isinstance(q, RaBitQuantizer):
        return dict(qtype=np.array("rabitq"), metric_type=np.array(int(q.metric_type)), d=np.array(q.rabitq.d))
    raise ValueError(f"save(): unsupported quantizer {type(q).__name__}")


def quantizer_from_state(z) -> BaseQuantizer:
    """Inverse of quantizer_state (z: a mapping of numpy arrays, e.g. an open .npz)."""
    qt = str(z["qtype"])
    if qt == "pq":
        q = ProductQuantizer(M=int(z["M"]), B=int(z["B"]))
        q.set_codebooks(z["centroids"])
    elif qt == "opq":
        q = OptimizedProductQuantizer(M=int(z["M"]), B=int(z["B"]))
        q.opq = OPQHandle(_arrays.to_device(z["A"]))
        inner = ProductQuantizer(M=int(z["M"]), B=int(z["B"]))
        inner.set_codebooks(z["centroids"])
        q._inner = inner
        q.pq = inner.pq
    elif qt == "sq":
        q = ScalarQuantizer(num_bits=int(z["num_bits"]))
        q.min = np.array(z["min"])
        q.max = np.array(z["max"])
    elif qt == "rabitq":
        from ...utils.faiss_utils import MetricType
        q = RaBitQuantizer(metric_type=MetricType(int(z["metric_type"])))
        q.fit(np.empty((0, int(z["d"])), dtype=np.float32))
    else:
        raise ValueError(f"load(): unknown quantizer type {qt!r}")
    return q


class FlatQuantizedIndex(BaseSearchIndex):
    """Brute-force search over the codes of any BaseQuantizer (GPU ADC for PQ / OPQ)."""

    def __init__(self, quantizer: BaseQuantizer) -> None:
        self._quantizer = quantizer
        self._codes: Optional[torch.Tensor] = None
        self._metric: Literal["l2", "ip"] = "l2"
        self._N = 0
        self._D = 0

    @property
    def quantizer(self) -> BaseQuantizer:
        return self._quantizer

    def fit(self, X, metric: Literal["l2", "ip"] = "l2") -> None:
        if metric not in _METRIC:
            raise ValueError(f"metric must be 'l2' or 'ip', got {metric!r}")
        Xd = _arrays.to_device(X, torch.float32)
        self._metric = metric
        self._N, self._D = Xd.shape
        self._quantizer.fit(Xd)
        self._codes = self._quantizer.compress(Xd)

    def search(self, Q, k: int) -> np.ndarray:
        ids, _ = self.search_with_scores(Q, k)
        return ids

    def search_with_scores(self, Q, k: int) -> Tuple[np.ndarray, np.ndarray]:
        Q = np.ascontiguousarray(Q, dtype=np.float32) if not _arrays.is_tensor(Q) else Q
        nq = Q.shape[0]
        k = min(int(k), self._N)
        if k <= 0:
            return np.empty((nq, 0), dtype=np.uint32), np.empty((nq, 0), dtype=np.float32)
        d, i = search_codes(self._quantizer, self._codes, Q, k, self._metric)
        return ids_to_numpy(i), _arrays.to_host(d)

    def memory_footprint(self) -> int:
        return int(self._codes.numel() * self._codes.element_size()) if self._codes is not None else 0

    def reconstruction_mse(self, X, sample_ids: Optional[np.ndarray] = None) -> Optional[float]:
        if self._codes is None:
            return None
        X = np.asarray(X, dtype=np.float32)
        if sample_ids is None:
            sample_ids = np.arange(self._N)
        ids = torch.from_numpy(np.asarray(sample_ids, dtype=np.int64)).to(self._codes.device)
        xh = self._quantizer.decompress(self._codes[ids].contiguous())
        xh = _arrays.to_host(xh).astype(np.float32)
        return float(np.mean((X[np.asarray(sample_ids)] - xh) ** 2))

    # --------------------------------------------------------------- persistence
    def _state(self) -> dict:
        st = {"codes": _arrays.to_host(self._codes), "metric": np.array(self._metric),
              "N": np.array(self._N), "D": np.array(self._D)}
        st.update(quantizer_state(self._quantizer))
        return st

    def save(self, path: str | Path) -> None:
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        with open(path, "wb") as f:
            np.savez(f, **self._state())

    def load(self, path: str | Path) -> None:
        with np.load(Path(path), allow_pickle=False) as z:
            q = quantizer_from_state(z)
            self._quantizer = q
            self._codes = torch.from_numpy(np.array(z["codes"])).to(_arrays.device())
            self._metric = str(z["metric"])
            self._N = int(z["N"])
            self._D = int(z["D"])


class FlatADCIndex(FlatQuantizedIndex):
    """FlatQuantizedIndex restricted to PQ / OPQ codes (pure LUT-sum ADC search)."""

    def __init__(self, quantizer: BaseQuantizer) -> None:
        if not isinstance(quantizer, (ProductQuantizer, OptimizedProductQuantizer)):
            raise ValueError("FlatADCIndex needs a ProductQuantizer or OptimizedProductQuantizer")
        super().__init__(quantizer)
