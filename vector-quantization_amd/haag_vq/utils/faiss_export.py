"""Codebook export and the codebook-query QPS proxy, without faiss.

Same module path and public functions as /root/reference/src/haag_vq/utils/faiss_export.py:
``write_fvecs`` / ``write_ivecs`` / ``load_fvecs`` / ``load_ivecs`` (:46-133, the faiss
.fvecs/.ivecs formats), ``export_codebook`` (:304-347) and ``query_codebook`` (:417-506)
with its per-subspace PQ path (``_query_product_codebook``, :352-414: for PQ / OPQ the
returned indices of subspace m are offset by m * ksub).  The searches run on the MI355X:
top-1 per subspace is the canonical PQ encode of the queries (``mivq_pq_encode``); other
top-k and flat codebooks use ``mivq_flat_search``.
"""

from __future__ import annotations

import math
from pathlib import Path
from typing import Optional, Tuple, Union

import numpy as np
import torch

from .. import _arrays, _native
from .faiss_utils import MetricType

PathLike = Union[str, Path]
METRIC_L2 = int(MetricType.L2)
METRIC_INNER_PRODUCT = int(MetricType.INNER_PRODUCT)


def _is_pq_like(model) -> bool:
    return hasattr(model, "codebooks") or hasattr(model, "pq")


def _is_opq(model) -> bool:
    return hasattr(model, "opq") and hasattr(model, "pq")


def _is_scalar(model) -> bool:
    return hasattr(model, "min") and hasattr(model, "max")


def _is_rabit(model) -> bool:
    return type(model).__name__ == "RaBitQuantizer"


# ------------------------------------------------------------------------------ vec files
def write_fvecs(path: PathLike, vectors: np.ndarray) -> Path:
    path = Path(path)
    v = np.asarray(vectors, dtype=np.float32)
    if v.ndim != 2:
        raise ValueError("fvecs expects a 2D array")
    rec = np.empty((v.shape[0], v.shape[1] + 1), dtype=np.float32)
    rec[:, 0] = np.array([v.shape[1]], dtype=np.int32).view(np.float32)[0]
    rec[:, 1:] = v
    path.write_bytes(rec.tobytes())
    return path


def write_ivecs(path: PathLike, vectors: np.ndarray) -> Path:
    path = Path(path)
    v = np.asarray(vectors, dtype=np.int32)
    if v.ndim != 2:
        raise ValueError("ivecs expects a 2D array")
    rec = np.empty((v.shape[0], v.shape[1] + 1), dtype=np.int32)
    rec[:, 0] = v.shape[1]
    rec[:, 1:] = v
    path.write_bytes(rec.tobytes())
    return path


def _load_vec_file(path: PathLike, value_dtype) -> np.ndarray:
    path = Path(path)
    if not path.exists():
        raise FileNotFoundError(path)
    raw = path.read_bytes()
    if not raw:
        return np.empty((0, 0), dtype=value_dtype)
    ints = np.frombuffer(raw, dtype=np.int32)
    dim = int(ints[0])
    if dim <= 0:
        raise ValueError(f"Invalid vector dimension ({dim}) in {path}")
    rec = dim + 1
    if ints.size % rec != 0:
        raise ValueError(f"Corrupt vector file: {path}")
    n = ints.size // rec
    if not np.all(ints.reshape(n, rec)[:, 0] == dim):
        raise ValueError(f"Non-uniform dimensions in {path}")
    if value_dtype == np.int32:
        return np.array(ints.reshape(n, rec)[:, 1:], copy=True)
    return np.array(np.frombuffer(raw, dtype=np.float32).reshape(n, rec)[:, 1:], copy=True)


def load_fvecs(path: PathLike) -> np.ndarray:
    return _load_vec_file(path, np.float32)


def load_ivecs(path: PathLike) -> np.ndarray:
    return _load_vec_file(path, np.int32)


# ------------------------------------------------------------------------------ export
def _extract_codebook(model) -> np.ndarray:
    if _is_opq(model) and not hasattr(model, "codebooks"):
        inner = model.inner
        return np.concatenate([np.asarray(c, np.float32) for c in inner.codebooks], axis=0)
    if _is_pq_like(model) and getattr(model, "codebooks", None):
        return np.concatenate([np.asarray(c, np.float32) for c in model.codebooks], axis=0)
    if _is_scalar(model):
        if model.min is None or model.max is None:
            raise ValueError("ScalarQuantizer must be fitted before exporting")
        return np.stack([model.min, model.max]).astype(np.float32)
    raise ValueError(f"Cannot export a codebook for {type(model).__name__}")


def export_codebook(model, output_dir: PathLike, *, index_key: Optional[str] = None, codes: Optional[np.ndarray] = None,
                    codebook_filename: str = "codebook.fvecs", codes_filename: str = "codes.ivecs") -> dict:
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    cb = _extract_codebook(model)
    result = {"codebook": write_fvecs(out / codebook_filename, cb), "codebook_vectors": cb}
    if codes is not None:
        result["codes"] = write_ivecs(out / codes_filename, np.asarray(codes, dtype=np.int32))
    return result


# ------------------------------------------------------------------------------ query
def _query_product_codebook(queries: np.ndarray, model, codebook_vectors: np.ndarray, topk: int,
                            metric: int) -> Tuple[np.ndarray, np.ndarray]:
    if _is_opq(model) and not hasattr(model, "codebooks"):
        inner = model.inner
        chunk_dim, M, ksub = int(inner.chunk_dim), int(model.M), 1 << int(model.B)
        q = model.opq.apply(queries)
    else:
        chunk_dim = int(model.chunk_dim)
        M = int(getattr(model, "M", getattr(model, "num_chunks", 0)))
        ksub = int(2 ** int(getattr(model, "B", int(round(math.log2(getattr(model, "num_clusters")))))))
        q = queries
    if codebook_vectors.shape != (M * ksub, chunk_dim):
        raise ValueError(
            "ProductQuantizer codebook has unexpected shape; expected "
            f"({M * ksub}, {chunk_dim}) but received {codebook_vectors.shape}"
        )
    if q.shape[1] != chunk_dim * M:
        raise ValueError(f"Query dimensionality does not match ProductQuantizer. Expected {chunk_dim * M} "
                         f"but received {q.shape[1]}")
    per = min(topk, ksub)
    if metric not in (METRIC_L2, METRIC_INNER_PRODUCT):
        raise ValueError("ProductQuantizer queries currently support only METRIC_L2 and METRIC_INNER_PRODUCT")
    qd = _arrays.to_device(q)
    C = _arrays.to_device(codebook_vectors).reshape(M, ksub, chunk_dim).contiguous()
    nq = qd.shape[0]
    nbits = int(round(math.log2(ksub)))
    if per == 1 and metric == METRIC_L2 and (ksub & (ksub - 1)) == 0:
        prep = _native.pq_prepare(C, nbits)
        codes = _native.pq_encode(qd, C, prep, nbits)
        u8 = codes if nbits == 8 else _native.pq_unpack(codes, M, nbits)
        lut = _native.adc_lut(qd, C, nbits, METRIC_L2)
        idx = u8.long()
        dist = torch.gather(lut, 2, idx.unsqueeze(-1)).squeeze(-1)
        offs = torch.arange(M, device=qd.device, dtype=torch.int64) * ksub
        return _arrays.to_host(dist), _arrays.to_host(idx + offs)
    dists = np.empty((nq, M * per), np.float32)
    ids = np.empty((nq, M * per), np.int64)
    for m in range(M):
        qm = qd[:, m * chunk_dim:(m + 1) * chunk_dim].contiguous()
        d, i = _native.flat_search(qm, C[m].contiguous(), per, metric)
        d = -d if metric == METRIC_INNER_PRODUCT else d
        dists[:, m * per:(m + 1) * per] = _arrays.to_host(d)
        ids[:, m * per:(m + 1) * per] = _arrays.to_host(i).view(np.uint32).astype(np.int64) + m * ksub
    return dists, ids


def query_codebook(queries, *, model=None, codebook_vectors: Optional[np.ndarray] = None,
                   codebook_path: Optional[PathLike] = None, topk: int = 1, metric: int = METRIC_L2,
                   index_key: Optional[str] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Nearest codebook entries of each query (faiss_export.py:417-506 semantics)."""
    if codebook_vectors is None:
        if codebook_path is None:
            raise ValueError("Provide either codebook_vectors or codebook_path")
        codebook_vectors = load_fvecs(codebook_path)
    codebook_vectors = np.ascontiguousarray(codebook_vectors, dtype=np.float32)
    if codebook_vectors.ndim != 2:
        raise ValueError("Codebook vectors must be 2D")
    queries = np.asarray(queries, dtype=np.float32)
    if queries.ndim == 1:
        queries = queries.reshape(1, -1)
    if queries.ndim != 2:
        raise ValueError("Queries must be a 1D or 2D array")
    if queries.size == 0:
        raise ValueError("No queries provided for search")
    if topk <= 0:
        raise ValueError("topk must be positive")
    if model is not None and (_is_pq_like(model) or _is_opq(model)) and not _is_scalar(model):
        return _query_product_codebook(queries, model, codebook_vectors, int(topk), int(metric))
    n_entries, dim = codebook_vectors.shape
    if n_entries == 0:
        raise ValueError("Codebook is empty; cannot run queries")
    if queries.shape[1] != dim:
        raise ValueError(f"Query dimensionality ({queries.shape[1]}) does not match codebook ({dim})")
    k = min(int(topk), n_entries)
    if int(metric) not in (METRIC_L2, METRIC_INNER_PRODUCT):
        raise ValueError("Provide a quantizer model to build complex indexes")
    d, i = _native.flat_search(_arrays.to_device(queries), _arrays.to_device(codebook_vectors), k, int(metric))
    if int(metric) == METRIC_INNER_PRODUCT:
        d = -d
    return _arrays.to_host(d), _arrays.to_host(i).view(np.uint32).astype(np.int64)
