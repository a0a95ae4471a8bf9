"""Dataset container and offline loaders.

``Dataset`` keeps the reference's contract (/root/reference/src/haag_vq/data/datasets.py:36-81):
queries default to the first ``num_queries`` vectors, ground truth is the exact L2 top-100
of the queries over the vectors (here: ``mivq_flat_search`` on the device, f32 like the
reference's faiss IndexFlatL2).  ``load_dummy_dataset`` reproduces
``np.random.seed(seed); np.random.randn(n, d)`` exactly (the fixture of the logged KATs).
The Hugging Face loaders need the network and are out of scope; ``load_local_dataset``
reads a local .npy / .fvecs file instead.
"""

from __future__ import annotations

import os
from pathlib import Path
from typing import Callable, Optional

import numpy as np


def compute_ground_truth(queries: np.ndarray, vectors: np.ndarray, k: int = 100) -> np.ndarray:
    """Exact L2 top-k ids (int64) of each query over the vectors, on the GPU."""
    from haag_vq import _arrays, _native

    k = min(k, len(vectors))
    _, ids = _native.flat_search(_arrays.to_device(np.asarray(queries, np.float32)),
                                 _arrays.to_device(np.asarray(vectors, np.float32)), k, _native.METRIC_L2)
    return _arrays.to_host(ids).view(np.uint32).astype(np.int64)


compute_ground_truth_faiss = compute_ground_truth  # reference name (datasets.py:8)


class Dataset:
    def __init__(self, vectors: np.ndarray, queries: Optional[np.ndarray] = None,
                 ground_truth: Optional[np.ndarray] = None, num_queries: int = 100,
                 distance_metric: Optional[Callable] = None, skip_ground_truth: bool = False):
        self.vectors = vectors
        if queries is None:
            self.queries = vectors[:num_queries]
        else:
            assert num_queries <= len(queries)
            self.queries = queries[:num_queries]
        if ground_truth is not None:
            assert num_queries <= len(ground_truth)
            self.ground_truth = ground_truth[:num_queries]
        elif skip_ground_truth:
            self.ground_truth = None
        else:
            self.ground_truth = compute_ground_truth(self.queries, self.vectors, k=100)
        self.distance_metric = distance_metric


def load_dummy_dataset(num_samples=10000, dim=1024, seed=42) -> Dataset:
    np.random.seed(seed)
    return Dataset(np.random.randn(num_samples, dim))


def _read_vectors(path: Path) -> np.ndarray:
    if path.suffix == ".npy":
        return np.load(path, allow_pickle=False)
    if path.suffix == ".fvecs":
        from haag_vq.utils.faiss_export import load_fvecs
        return load_fvecs(path)
    raise ValueError(f"unsupported vector file {path} (use .npy or .fvecs)")


def load_local_dataset(path, limit: Optional[int] = None, num_queries: int = 100) -> Dataset:
    X = _read_vectors(Path(path))
    if limit is not None:
        X = X[:limit]
    return Dataset(np.ascontiguousarray(X, dtype=np.float32), num_queries=num_queries)


def load_dbpedia_openai_1536_100k(limit: Optional[int] = None, cache_dir: str = "../datasets") -> Dataset:
    """dbpedia-100k (1536-d) from a local file: $VQ_DATA_DIR/dbpedia-100k.{npy,fvecs}."""
    root = Path(os.environ.get("VQ_DATA_DIR", cache_dir))
    for name in ("dbpedia-100k.npy", "dbpedia-100k.fvecs", "dbpedia_100k.npy", "dbpedia_100k.fvecs"):
        if (root / name).exists():
            return load_local_dataset(root / name, limit=limit)
    raise FileNotFoundError(
        f"dbpedia-100k is fetched from the Hugging Face Hub by the reference; offline, place "
        f"dbpedia-100k.npy or .fvecs under {root} (or set VQ_DATA_DIR)"
    )
