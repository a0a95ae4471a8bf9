"""Rank distortion@k = 1 - recall@k — /root/reference/src/haag_vq/metrics/rank_distortion.py:47-144."""

import numpy as np

from .recall import retrieve


def compute_rank_distortion(data, model, k: int = 10, num_queries: int = 100) -> float:
    true_top = data.ground_truth[:num_queries, :k]
    got = retrieve(data, model, k=k, num_queries=num_queries)
    missing = 0
    for i in range(len(true_top)):
        missing += len(set(np.asarray(true_top[i]).tolist()) - set(got[i, :k].tolist()))
    return float(missing / (len(true_top) * k))


def compute_rank_distortion_per_query(data, model, k: int = 10, num_queries: int = 100) -> np.ndarray:
    true_top = data.ground_truth[:num_queries, :k]
    got = retrieve(data, model, k=k, num_queries=num_queries)
    out = np.zeros(len(true_top))
    for i in range(len(true_top)):
        out[i] = len(set(np.asarray(true_top[i]).tolist()) - set(got[i, :k].tolist())) / k
    return out
