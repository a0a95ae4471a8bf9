"""Recall@k — /root/reference/src/haag_vq/metrics/recall.py:6-43.

``evaluate_recall`` re-encodes the database (as the reference does) and ranks it for the
first ``num_queries`` queries.  With the dataset's default metric (sklearn
``pairwise_distances``, Euclidean — its ranking is the squared-L2 ranking) the ranking runs
on the MI355X (ADC for PQ / OPQ, decode + exact search otherwise; see
methods/search/flat_quantized_index.py) instead of a full numpy argsort.  Any other
``data.distance_metric`` is honoured as upstream does (recall.py:14): decode, call the
metric on (queries, reconstructions), argsort on the host.
"""

import numpy as np

from haag_vq.data.datasets import is_euclidean
from haag_vq.methods.search.flat_quantized_index import ids_to_numpy, search_codes


def retrieve(data, model, k: int, num_queries: int = 100) -> np.ndarray:
    codes = model.compress(data.vectors)  # the dataset's own dtype, as the reference (recall.py:12)
    k = min(k, len(data.vectors))
    metric = getattr(data, "distance_metric", None)
    if not is_euclidean(metric):
        rec = model.decompress(codes)
        if not isinstance(rec, np.ndarray):
            rec = rec.detach().cpu().numpy()
        dists = np.asarray(metric(data.queries[:num_queries], rec))
        return dists.argsort(axis=1, kind="stable")[:, :k].astype(np.int64)
    queries = np.asarray(data.queries[:num_queries], dtype=np.float32)
    _, ids = search_codes(model, codes, queries, k, "l2")
    return ids_to_numpy(ids).astype(np.int64)


def evaluate_recall(data, model, num_queries=100):
    true_nn = data.ground_truth[:num_queries]
    retrieved = retrieve(data, model, k=100, num_queries=num_queries)
    return {
        "recall@10": recall_at_k(true_nn, retrieved, k=10),
        "recall@100": recall_at_k(true_nn, retrieved, k=100),
    }


def recall_at_k(true_nn: np.ndarray, retrieved: np.ndarray, k: int) -> float:
    """Mean over queries of |gt[:k] & retrieved[:k]| / k."""
    hits = 0
    for i in range(len(true_nn)):
        hits += len(set(np.asarray(true_nn[i, :k]).tolist()) & set(np.asarray(retrieved[i, :k]).tolist())) / k
    return hits / len(true_nn)
