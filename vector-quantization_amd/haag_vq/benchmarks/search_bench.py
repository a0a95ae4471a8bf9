"""Benchmark harness for ``BaseSearchIndex`` implementations: recall@k, QPS (best of a few
timed searches), memory footprint / compression and reconstruction MSE per index, plus the
bpd sweep and the method comparison that tabulate them.

Mirrors /root/reference/src/haag_vq/benchmarks/search_bench.py:25-218.  Ground truth comes from
``mivq_flat_search`` on the device (the reference builds a faiss IndexFlatL2 / IndexFlatIP);
the indexes themselves (``FlatQuantizedIndex``, ``FaissIvfPqIndex``, ``RaBitQIndex``) search on
the MI355X path.  ``pareto_plot`` needs matplotlib, which this image does not ship.
"""

from __future__ import annotations

import time
from datetime import datetime, timezone
from typing import Callable, Dict, Optional

import numpy as np
import pandas as pd

from haag_vq.methods.base_search_index import BaseSearchIndex


def _utc_timestamp() -> str:
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def compute_ground_truth(X_train: np.ndarray, X_query: np.ndarray, k: int = 10, metric: str = "l2") -> np.ndarray:
    """(nq, min(k, N)) int64 ids of the exact nearest rows (L2) or largest inner products ('ip'),
    best first, from ``mivq_flat_search``."""
    from haag_vq import _arrays, _native

    X = np.ascontiguousarray(X_train, dtype=np.float32)
    Qh = np.ascontiguousarray(X_query, dtype=np.float32)
    k = min(int(k), X.shape[0])
    m = _native.METRIC_INNER_PRODUCT if metric == "ip" else _native.METRIC_L2
    if k == 0 or Qh.shape[0] == 0:
        return np.empty((Qh.shape[0], k), dtype=np.int64)
    _, ids = _native.flat_search(_arrays.to_device(Qh), _arrays.to_device(X), k, metric=m)
    return _arrays.to_host(ids).view(np.uint32).astype(np.int64)


def _compute_recall(ids: np.ndarray, ground_truth: np.ndarray, k: int) -> float:
    """Hits of the returned top-k among the true top-k, summed over queries, over nq * k_gt."""
    k_gt = min(k, ground_truth.shape[1])
    k_ret = min(k, ids.shape[1])
    total = ids.shape[0] * k_gt
    if total == 0:
        return 0.0
    hits = sum(len(set(g[:k_gt].tolist()).intersection(r[:k_ret].tolist())) for g, r in zip(ground_truth, ids))
    return hits / total


def benchmark_index(index: BaseSearchIndex, X_train: np.ndarray, X_query: np.ndarray, gt_ids: np.ndarray,
                    k: int = 10, repeats: int = 3, mse_sample: int = 1000) -> Dict:
    """Fit, then ``repeats`` timed searches: the fastest sets the QPS and supplies the ids the
    recall is computed on; memory footprint vs raw float32, MSE on a seed-0 row sample."""
    X = np.ascontiguousarray(X_train, dtype=np.float32)
    Qh = np.ascontiguousarray(X_query, dtype=np.float32)
    N, D = X.shape
    index.fit(X)
    best_t, best_ids = float("inf"), None
    for _ in range(repeats):
        t0 = time.perf_counter()
        got = index.search(Qh, k)  # returns host arrays: the device work is complete
        dt = time.perf_counter() - t0
        if dt < best_t:
            best_t, best_ids = dt, got
    mem = index.memory_footprint()
    sample = (np.arange(N, dtype=np.uint32) if N <= mse_sample
              else np.random.default_rng(0).choice(N, mse_sample, replace=False).astype(np.uint32))
    return {
        "method": type(index).__name__,
        "recall_at_k": _compute_recall(np.asarray(best_ids), gt_ids, k),
        "qps": Qh.shape[0] / best_t if best_t > 0 else float("inf"),
        "memory_bytes": mem,
        "compression_ratio": (N * D * 4) / mem if mem > 0 else float("inf"),
        "mse": index.reconstruction_mse(X, sample_ids=sample),
        "k": k,
        "N": N,
        "D": D,
    }


def sweep_bpd(index_factory: Callable[[float], BaseSearchIndex], bpd_values: list, X_train: np.ndarray,
              X_query: np.ndarray, gt_ids: np.ndarray, k: int = 10) -> pd.DataFrame:
    """One row per bpd (the factory builds an unfitted index for it); one timestamp per sweep."""
    stamp = _utc_timestamp()
    rows = []
    for bpd in bpd_values:
        r = benchmark_index(index_factory(bpd), X_train, X_query, gt_ids, k=k)
        r.update(bpd=bpd, timestamp=stamp)
        rows.append(r)
    return pd.DataFrame(rows)


def compare_methods(method_configs: Dict[str, BaseSearchIndex], X_train: np.ndarray, X_query: np.ndarray,
                    gt_ids: np.ndarray, k: int = 10) -> pd.DataFrame:
    """One row per named (unfitted) index; the name replaces the class name in 'method'."""
    stamp = _utc_timestamp()
    rows = []
    for name, index in method_configs.items():
        r = benchmark_index(index, X_train, X_query, gt_ids, k=k)
        r.update(method=name, timestamp=stamp)
        rows.append(r)
    return pd.DataFrame(rows)


def pareto_plot(df: pd.DataFrame, x: str = "compression_ratio", y: str = "recall_at_k", hue: str = "method",
                save_path: Optional[str] = None) -> None:
    """Recall-vs-compression scatter, one series per ``hue`` value (needs matplotlib)."""
    try:
        import matplotlib.pyplot as plt
    except ImportError as e:  # not in this image; plotting is a report step
        raise ImportError("pareto_plot needs matplotlib") from e
    fig, ax = plt.subplots(figsize=(8, 5))
    for name, grp in df.groupby(hue):
        ax.scatter(grp[x], grp[y], label=str(name), s=80)
        ax.plot(grp[x], grp[y], linewidth=1, alpha=0.6)
    ax.set_xlabel(x)
    ax.set_ylabel(y)
    ax.set_title(f"Pareto: {y} vs {x}")
    ax.legend(loc="lower right", fontsize=7)
    fig.tight_layout()
    if save_path is None:
        plt.show()
    else:
        fig.savefig(save_path, dpi=150, bbox_inches="tight")
        plt.close(fig)
