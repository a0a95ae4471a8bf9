"""`vq-benchmark ivf-bench`: method runners over a ``train.npy`` / ``queries.npy`` directory at a
bits-per-dimension budget, one CSV row per method.

Mirrors /root/reference/src/haag_vq/benchmarks/ivf_benchmark.py:32-455 (the
``pq_flat`` / ``opq_flat`` / ``sq_flat`` runners are on the hot path).  Same options, runner
names, bpd rules, recall definition, CSV columns and timestamped output name.  What runs where:

* ``pq_flat`` / ``opq_flat`` / ``sq_flat`` (reference :95-167, :272-310): fit, encode all rows
  (``mivq_pq_encode`` / OPQ rotation + encode / ``mivq_sq_encode``), decode, then the exact L2
  top-k of the queries over the reconstructions with ``mivq_flat_search`` — the reference adds
  the reconstructions to a faiss ``IndexFlatL2``; both are exact searches over the same rows.
  The data stay on the device from encode to search; the timed region is the search, as in the
  reference (``index.search`` only).  The MSE is the mean over rows of the squared
  reconstruction error, summed in fp64 on the device (the reference sums in fp32 numpy).
* ``faiss_ivfpq`` (reference :170-204): the device IVF-PQ index (``FaissIvfPqIndex``: coarse
  k-means, residual PQ, ADC over ``nprobe`` lists) with the reference's factory parameters
  ``IVF{nlist},PQ{M}x8`` and its memory formula.
* ``rabitq`` (reference :207-240): ``RaBitQIndex`` (``mivq_rabitq_search``).
* ``rabitq_ivf`` and ``saq`` (reference :243-269, :313-348) are not part of the MI355X build
  (DESIGN.md §9): they are reported and skipped like an unknown method.

Ground truth, when the directory has no ``ground_truth.npy``, is the exact L2 top-``gt_k`` from
``mivq_flat_search`` (the reference: faiss ``IndexFlatL2``) and is saved there for reuse, as
the reference does.  faiss is not needed.
"""

from __future__ import annotations

import csv
from datetime import datetime, timezone
from pathlib import Path
from time import perf_counter
from typing import Dict, Optional

import numpy as np
import typer

NOT_IN_BUILD = ("rabitq_ivf", "saq")


def _load_npy_dataset(dataset_dir: str, num_queries: int = 1000):
    """(train, queries, gt or None) — reference :32-57: without ``queries.npy`` the last
    ``num_queries`` rows of ``train.npy`` become the queries."""
    d = Path(dataset_dir)
    train_path, queries_path, gt_path = d / "train.npy", d / "queries.npy", d / "ground_truth.npy"
    if not train_path.exists():
        raise FileNotFoundError(f"train.npy not found in {d}")
    train = np.load(train_path).astype(np.float32)
    if queries_path.exists():
        queries = np.load(queries_path).astype(np.float32)
    else:
        queries = train[-num_queries:]
        train = train[:-num_queries]
    gt = np.load(gt_path) if gt_path.exists() else None
    return train, queries, gt


def _compute_ground_truth(train: np.ndarray, queries: np.ndarray, k: int) -> np.ndarray:
    """Exact L2 k-NN ids (nq, k) on the device (reference :60-67 uses faiss IndexFlatL2)."""
    from .precompute_ground_truth import exact_knn_l2

    return exact_knn_l2(train, queries, k)[0]


def _recall_at_k(gt: np.ndarray, retrieved: np.ndarray, k: int) -> float:
    """Fraction of the true top-k found in the retrieved top-k (reference :70-78)."""
    nq = gt.shape[0]
    hits = 0
    for i in range(nq):
        hits += len(set(gt[i, :k].tolist()) & set(retrieved[i, :k].tolist()))
    return hits / (nq * k)


def _bpd_to_pq_M(D: int, bpd: int) -> int:
    """PQ subquantizers for a bits-per-dimension budget at 8 bits per code (reference :81-92):
    M = D * bpd // 8, at least 1, lowered until it divides D."""
    M = max(1, D * bpd // 8)
    while D % M != 0 and M > 1:
        M -= 1
    return M


def _nbytes(codes) -> int:
    if isinstance(codes, np.ndarray):
        return int(codes.nbytes)
    return int(codes.numel() * codes.element_size())


def _flat_runner(name: str, model, train: np.ndarray, queries: np.ndarray, gt: np.ndarray, k: int) -> Dict:
    """The shared body of the three flat runners: fit, encode, decode, MSE, exact search over
    the reconstructions (timed), recall and memory."""
    import torch

    from haag_vq import _arrays, _native

    t0 = perf_counter()
    model.fit(train)
    print(f"  {name}: fit in {perf_counter() - t0:.1f}s")
    Xd = _arrays.to_device(train)
    codes = model.compress(Xd)
    rec = model.decompress(codes).float().contiguous()
    tot = torch.zeros((), dtype=torch.float64, device=rec.device)
    for s in range(0, rec.shape[0], 1 << 18):  # fp64 per row slice (bounded scratch)
        tot += (Xd[s:s + (1 << 18)].double() - rec[s:s + (1 << 18)].double()).pow(2).sum()
    mse = float(tot.item()) / max(rec.shape[0], 1)
    del Xd
    if k > 256:
        raise ValueError(f"k={k} > 256: the flat search keeps at most 256 per query")
    Qd = _arrays.to_device(queries)
    torch.cuda.synchronize()
    t0 = perf_counter()
    _, ids = _native.flat_search(Qd, rec, min(k, rec.shape[0]))
    retrieved = _arrays.to_host(ids).view(np.uint32).astype(np.int64)  # waits for the search
    search_time = perf_counter() - t0
    mem = _nbytes(codes)
    return {
        "recall_at_k": _recall_at_k(gt, retrieved, k),
        "qps": len(queries) / max(search_time, 1e-12),
        "memory_bytes": mem,
        "compression_ratio": train.nbytes / max(mem, 1),
        "mse": mse,
    }


def _run_pq_flat(train, queries, gt, k, bpd):
    """PQ (B = 8, M from the bpd budget) with exact search on the reconstructions (reference :95-131)."""
    from haag_vq.methods.product_quantization import ProductQuantizer

    return _flat_runner("pq_flat", ProductQuantizer(M=_bpd_to_pq_M(train.shape[1], bpd), B=8), train, queries, gt, k)


def _run_sq_flat(train, queries, gt, k, bpd):
    """SQ at bpd bits when bpd is 4, 8 or 16, else 8 (reference :134-167)."""
    from haag_vq.methods.scalar_quantization import ScalarQuantizer

    num_bits = bpd if bpd in (4, 8, 16) else 8
    return _flat_runner("sq_flat", ScalarQuantizer(num_bits=num_bits), train, queries, gt, k)


def _run_opq_flat(train, queries, gt, k, bpd):
    """OPQ (rotation + PQ, B = 8) with exact search on the reconstructions (reference :272-310)."""
    from haag_vq.methods.optimized_product_quantization import OptimizedProductQuantizer

    model = OptimizedProductQuantizer(M=_bpd_to_pq_M(train.shape[1], bpd), B=8)
    return _flat_runner("opq_flat", model, train, queries, gt, k)


def _run_faiss_ivfpq(train, queries, gt, k, bpd, K, nprobe):
    """IVF{K},PQ{M}x8 on the device: train, add, search (reference :170-204)."""
    from haag_vq.methods.search.faiss_ivfpq_index import FaissIvfPqIndex

    D = train.shape[1]
    M = _bpd_to_pq_M(D, bpd)
    print(f"  faiss_ivfpq: IVF{K},PQ{M}x8, nprobe={nprobe}")
    index = FaissIvfPqIndex(K=K, m=M, nbits=8, nprobe=nprobe)
    t0 = perf_counter()
    index.fit(train)
    print(f"  faiss_ivfpq: index built in {perf_counter() - t0:.1f}s")
    t0 = perf_counter()
    retrieved = index.search(queries, k)
    search_time = perf_counter() - t0
    mem = train.shape[0] * M + K * D * 4  # the reference's estimate: codes + coarse centroids
    return {
        "recall_at_k": _recall_at_k(gt, retrieved, k),
        "qps": len(queries) / max(search_time, 1e-12),
        "memory_bytes": mem,
        "compression_ratio": train.nbytes / max(mem, 1),
        "mse": "",
    }


def _run_rabitq(train, queries, gt, k, bpd):
    """Flat RaBitQ with the estimator search; ``bpd`` is ignored (reference :207-240)."""
    from haag_vq.methods.search.rabitq_index import RaBitQIndex

    model = RaBitQIndex()
    t0 = perf_counter()
    model.fit(train)
    print(f"  rabitq: fit in {perf_counter() - t0:.1f}s")
    t0 = perf_counter()
    retrieved = model.search(queries, k)
    search_time = perf_counter() - t0
    mem = int(model.memory_footprint())
    mse = model.reconstruction_mse(train, sample_ids=np.arange(min(1000, len(train))))
    return {
        "recall_at_k": _recall_at_k(gt, retrieved, k),
        "qps": len(queries) / max(search_time, 1e-12),
        "memory_bytes": mem,
        "compression_ratio": train.nbytes / max(mem, 1),
        "mse": mse if mse is not None else "",
    }


METHOD_RUNNERS = {
    "pq_flat": lambda t, q, gt, k, bpd, K, np_: _run_pq_flat(t, q, gt, k, bpd),
    "opq_flat": lambda t, q, gt, k, bpd, K, np_: _run_opq_flat(t, q, gt, k, bpd),
    "sq_flat": lambda t, q, gt, k, bpd, K, np_: _run_sq_flat(t, q, gt, k, bpd),
    "faiss_ivfpq": _run_faiss_ivfpq,
    "rabitq": lambda t, q, gt, k, bpd, K, np_: _run_rabitq(t, q, gt, k, bpd),
}

FIELDNAMES = ["method", "recall_at_k", "qps", "memory_bytes", "compression_ratio", "mse", "k", "N", "D", "timestamp"]


def _utc_timestamp() -> str:
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def _timestamped_output_path(path: Path, now: Optional[datetime] = None) -> Path:
    """``name_YYYYMMDD_HHMMSS.suffix`` so that re-runs do not overwrite (reference :367-372)."""
    now = now or datetime.now(timezone.utc)
    return path.with_name(f"{path.stem}_{now.strftime('%Y%m%d_%H%M%S')}{path.suffix}")


def ivf_benchmark(
    dataset: str = typer.Option(..., help="Path to dataset directory containing train.npy and queries.npy"),
    methods: str = typer.Option("faiss_ivfpq,saq", help="Comma-separated methods: pq_flat,sq_flat,faiss_ivfpq,saq"),
    bpd: int = typer.Option(4, help="Bits per dimension budget"),
    k: int = typer.Option(10, help="Top-k for recall evaluation"),
    nlist: int = typer.Option(256, help="Number of IVF clusters"),
    nprobe: int = typer.Option(32, help="Number of IVF clusters to probe at search time"),
    output: str = typer.Option(..., help="Path to output CSV file"),
    num_queries: int = typer.Option(1000, help="Number of query vectors"),
    gt_k: int = typer.Option(100, help="k for ground truth computation (must be >= k)"),
) -> Optional[Path]:
    """Run the method runners on .npy datasets and write the CSV (returns its path)."""
    print(f"Loading dataset from {dataset}...")
    train, queries, gt = _load_npy_dataset(dataset, num_queries=num_queries)
    N, D = train.shape
    print(f"  train: {train.shape}, queries: {queries.shape}")
    if gt is None:
        print(f"Computing ground truth (k={gt_k})...")
        t0 = perf_counter()
        gt = _compute_ground_truth(train, queries, gt_k)
        print(f"  Ground truth computed in {perf_counter() - t0:.1f}s")
        gt_path = Path(dataset) / "ground_truth.npy"
        np.save(gt_path, gt)
        print(f"  Saved to {gt_path}")

    results = []
    run_ts = _utc_timestamp()
    for method_name in (m.strip() for m in methods.split(",")):
        runner = METHOD_RUNNERS.get(method_name)
        if runner is None:
            why = "not part of the MI355X build (DESIGN.md §9)" if method_name in NOT_IN_BUILD else "unknown"
            print(f"WARNING: method '{method_name}' is {why}, skipping. Available: {list(METHOD_RUNNERS)}")
            continue
        print(f"\nRunning {method_name} (bpd={bpd}, nlist={nlist}, nprobe={nprobe})...")
        try:
            metrics = runner(train, queries, gt, k, bpd, nlist, nprobe)
        except Exception as e:  # one failing method does not end the run (reference :432-435)
            print(f"  ERROR running {method_name}: {e}")
            import traceback

            traceback.print_exc()
            continue
        results.append({"method": method_name, "k": k, "N": N, "D": D, "timestamp": run_ts, **metrics})
        print(f"  recall@{k}={metrics['recall_at_k']:.4f}  qps={metrics['qps']:.1f}  "
              f"compression={metrics['compression_ratio']:.1f}x")

    if not results:
        print("\nNo results to write.")
        return None
    out_path = _timestamped_output_path(Path(output))
    out_path.parent.mkdir(parents=True, exist_ok=True)
    with open(out_path, "w", newline="") as f:
        writer = csv.DictWriter(f, fieldnames=FIELDNAMES)
        writer.writeheader()
        writer.writerows(results)
    print(f"\nResults written to {out_path}")
    return out_path


if __name__ == "__main__":
    typer.run(ivf_benchmark)
