"""The quantizer study: for every (method, bits per dimension) pair, fit a quantizer from the
registry, rank its scaled reconstructions against the queries by exact inner product, and tabulate
recall@k, reconstruction MSE and the compression factor.

Mirrors /root/reference/src/haag_vq/benchmarks/quantizer_study.py:37-150 (``run_study_arrays``,
``run_study``, ``main``): the second caller of ``build_quantizer`` and of
``FaissQuantizerAdapter`` next to ``vq-benchmark sweep``.  Every step runs on the MI355X path:
the quantizers encode / decode through libmivq, ``exact_search`` ranks with ``mivq_flat_search``.
"""

from __future__ import annotations

import argparse
from datetime import datetime, timezone
from pathlib import Path
from typing import Dict, List, Sequence, Tuple

import numpy as np
import pandas as pd

from haag_vq.benchmarks import exact_search as es
from haag_vq.benchmarks.study_config import StudyConfig, load_study_config


def _utc_now(fmt: str) -> str:
    return datetime.now(timezone.utc).strftime(fmt)


def _make_quantizer(method: str, bpd: float, D: int):
    from haag_vq.benchmarks.method_registry import build_quantizer

    return build_quantizer(method, bpd=bpd, D=D)


def _mse_rows(n: int, mse_sample: int) -> np.ndarray:
    """The rows the MSE is measured on: all of them, or a seed-0 sample without replacement."""
    if n <= mse_sample:
        return np.arange(n, dtype=np.uint32)
    return np.random.default_rng(0).choice(n, mse_sample, replace=False).astype(np.uint32)


def _study_row(q, method: str, bpd: float, X: np.ndarray, Q: np.ndarray, norms: np.ndarray, gt: np.ndarray,
               ks: Tuple[int, ...], chunk_size: int, sample: np.ndarray, stamp: str) -> Dict:
    n, D = X.shape
    q.fit(X)
    index = es.build_scaled_ip_index(q.reconstruct, n=n, d=D, norms=norms, chunk=chunk_size)
    _, ids = es.search_index(index, Q, k=max(ks))
    recalls = es.recall_at_ks(ids, gt, ks=ks)
    cb = q.code_bytes()
    out = {
        "method": method,
        "bpd": bpd,
        "compression_factor": (n * D * 4) / cb if cb else float("inf"),
        "code_bytes": cb,
        "mse": es.reconstruction_mse(X, q.reconstruct, sample, chunk=chunk_size),
        "n_db": n,
        "n_queries": Q.shape[0],
        "D": D,
        "timestamp": stamp,
    }
    out.update({f"recall_at_{k}": recalls[k] for k in ks})
    return out


def run_study_arrays(X: np.ndarray, Q: np.ndarray, methods: Sequence[str], bpd_values: Sequence[float],
                     ks: Tuple[int, ...] = (1, 10, 100), chunk_size: int = 50_000,
                     mse_sample: int = 100_000) -> pd.DataFrame:
    """One row per (method, bpd): ground truth is the exact normalised-IP top-max(ks) of the raw
    vectors, the candidate ranking that of x̂ / ‖x‖ (exact_search.py), MSE over a seed-0 sample."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    Q = np.ascontiguousarray(Q, dtype=np.float32)
    ks = tuple(int(k) for k in ks)
    stamp = _utc_now("%Y-%m-%dT%H:%M:%SZ")
    norms = es.compute_exact_norms(X)
    gt = es.normalized_ground_truth(X, Q, k=max(ks), norms=norms, chunk=chunk_size)
    sample = _mse_rows(X.shape[0], mse_sample)
    rows: List[Dict] = []
    for method in methods:
        for bpd in bpd_values:
            q = _make_quantizer(method, bpd, X.shape[1])
            rows.append(_study_row(q, method, bpd, X, Q, norms, gt, ks, chunk_size, sample, stamp))
            del q
    return pd.DataFrame(rows)


def _read_fvecs(path: str) -> np.ndarray:
    """``.fvecs``: per row an int32 dimension then that many float32 values."""
    raw = np.fromfile(path, dtype=np.float32)
    if raw.size == 0:
        raise ValueError(f"_load_fvecs: file is empty: {path}")
    d = int(raw[:1].view(np.int32)[0])
    if raw.size % (d + 1):
        raise ValueError(f"_load_fvecs: size {raw.size} floats not divisible by (d+1)={d + 1}: {path}")
    return raw.reshape(-1, d + 1)[:, 1:].copy()


_load_fvecs = _read_fvecs  # the reference's name


def run_study(config: StudyConfig) -> pd.DataFrame:
    ds = config.dataset
    X = _read_fvecs(ds["base_fvecs"])
    Q = _read_fvecs(ds["query_fvecs"])
    Q = Q[: int(ds.get("n_queries", Q.shape[0]))]
    df = run_study_arrays(X, Q, methods=config.methods, bpd_values=config.bpd, ks=tuple(config.ks),
                          chunk_size=config.chunk_size, mse_sample=config.mse_sample)
    df.insert(0, "dataset", ds.get("name", "unknown"))
    return df


def main(argv: List[str] | None = None) -> None:
    ap = argparse.ArgumentParser(description="VQ quantizer benchmark study")
    ap.add_argument("--config", required=True, help="Path to study YAML config")
    ap.add_argument("--plot", action="store_true", help="Also write Pareto plots")
    args = ap.parse_args(argv)
    cfg = load_study_config(args.config)
    df = run_study(cfg)
    out = Path(cfg.output_dir)
    out.mkdir(parents=True, exist_ok=True)
    stamp = _utc_now("%Y%m%d_%H%M%S")
    csv_path = out / f"results_{stamp}.csv"
    df.to_csv(csv_path, index=False)
    print(f"Saved results to {csv_path}")
    print(df.to_string(index=False))
    if args.plot:
        # the reference's study_plots (matplotlib Pareto curves) is a report script, out of scope
        # here; the CSV carries every plotted column
        print("--plot: Pareto plotting is not part of this build; the CSV holds the data")


if __name__ == "__main__":
    main()
