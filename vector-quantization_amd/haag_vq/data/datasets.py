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


def _default_metric():
    from sklearn.metrics import pairwise_distances  # the reference's default (datasets.py:43)

    return pairwise_distances


def is_euclidean(metric) -> bool:
    """True for the reference's default ranking metric (sklearn pairwise_distances, Euclidean):
    its ranking equals the squared-L2 ranking the device kernels compute."""
    if metric is None:
        return True
    try:
        from sklearn.metrics import pairwise_distances
    except ImportError:  # pragma: no cover
        return False
    return metric is pairwise_distances


class Dataset:
    def __init__(self, vectors: np.ndarray, queries: Optional[np.ndarray] = None,
                 ground_truth: Optional[np.ndarray] = None, num_queries: int = 100,
                 distance_metric: Optional[Callable] = None, skip_ground_truth: bool = False):
        if distance_metric is None:
            distance_metric = _default_metric()
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


# the reference's Hugging Face datasets (sweep.py:121-167) -> local file stems
_LOCAL_NAMES = {
    "dbpedia-100k": ("dbpedia-100k", "dbpedia_100k"),
    "dbpedia-1536": ("dbpedia-1536", "dbpedia_1536"),
    "dbpedia-3072": ("dbpedia-3072", "dbpedia_3072"),
    "cohere-msmarco": ("cohere-msmarco", "msmarco"),
    "huggingface": ("huggingface", "stsb_multi_mt"),
}
# upstream's default limits when none is given (sweep.py:131-160)
_DEFAULT_LIMIT = {"cohere-msmarco": 100_000, "dbpedia-1536": 100_000, "dbpedia-3072": 100_000}


def load_named_dataset(name: str, limit: Optional[int] = None, cache_dir: str = "../datasets") -> Dataset:
    """A dataset the reference downloads, read from $VQ_DATA_DIR (or cache_dir)/<name>.{npy,fvecs}."""
    if name not in _LOCAL_NAMES:
        raise ValueError(f"Unsupported dataset: {name}")
    root = Path(os.environ.get("VQ_DATA_DIR", cache_dir))
    for stem in _LOCAL_NAMES[name]:
        for ext in (".npy", ".fvecs"):
            if (root / f"{stem}{ext}").exists():
                return load_local_dataset(root / f"{stem}{ext}", limit=limit if limit is not None
                                          else _DEFAULT_LIMIT.get(name))
    raise FileNotFoundError(
        f"{name} is fetched from the Hugging Face Hub by the reference; offline, place "
        f"{_LOCAL_NAMES[name][0]}.npy or .fvecs under {root} (or set VQ_DATA_DIR)"
    )


def load_dbpedia_openai_1536_100k(limit: Optional[int] = None, cache_dir: str = "../datasets") -> Dataset:
    """dbpedia-100k (1536-d) from a local file: $VQ_DATA_DIR/dbpedia-100k.{npy,fvecs}."""
    return load_named_dataset("dbpedia-100k", limit=limit, cache_dir=cache_dir)
