"""Search-index benchmark driver: builds ``BaseSearchIndex`` objects per method name and runs the
``search_bench`` harness in compare mode (several methods at one bpd) or sweep mode (one
method over several bpd values).

Mirrors /root/reference/src/haag_vq/benchmarks/run_benchmarks.py:25-415 (SURVEY §2 row
``search_bench.py, run_benchmarks.py``: ``build_method_configs`` :118-246): the same dataset
formats (``train.npy`` + ``queries.npy`` [+ ``groundtruth.npy``], ``base.fvecs`` +
``query.fvecs`` [+ ``groundtruth.ivecs``], or ``synthetic``), the same method names and
parameter rules (M from the bpd budget at 8 bits per sub-code, SQ bit depth by bpd band, OPQ's
M lowered until it divides D), the same arguments and timestamped CSV.  The indexes search on
the MI355X path: ``FlatQuantizedIndex`` (PQ / OPQ by ADC, ``mivq_adc_search``; SQ by decode +
``mivq_flat_search``), ``FaissIvfPqIndex`` (device IVF-PQ), ``RaBitQIndex``
(``mivq_rabitq_search``); ground truth from ``mivq_flat_search``.  ``pq_ivf``, ``saq`` and
``rabitq_ivf`` are not part of the MI355X build: they are reported unavailable
and skipped, as the reference does for a method whose import fails.

usage: python -m haag_vq.benchmarks.run_benchmarks [--dataset synthetic] [--methods ...] [--bpd 8]
       [--sweep-bpd 2,4,8] [--k 10] [--output results.csv] [--K 1024] [--nprobe 64]
"""

from __future__ import annotations

import argparse
import sys
from datetime import datetime, timezone
from pathlib import Path
from typing import Optional

import numpy as np

from haag_vq.benchmarks.search_bench import compare_methods, compute_ground_truth, pareto_plot, sweep_bpd

AVAILABLE_METHODS = ("pq_flat", "opq_flat", "sq_flat", "pq_ivf", "faiss_ivfpq", "saq", "rabitq", "rabitq_ivf")
NOT_IN_BUILD = ("pq_ivf", "saq", "rabitq_ivf")


def load_dataset(dataset_path: str):
    """(X_train, X_query, gt ids or None) from a .npy or .fvecs directory, or ``synthetic``
    (2000 x 64 train, 100 queries, standard normal, seed 0) — reference :43-90."""
    from haag_vq.utils.faiss_export import load_fvecs, load_ivecs

    if dataset_path == "synthetic":
        rng = np.random.default_rng(0)
        return rng.standard_normal((2000, 64)).astype(np.float32), rng.standard_normal((100, 64)).astype(np.float32), None
    p = Path(dataset_path)
    if not p.exists():
        raise FileNotFoundError(f"Dataset path not found: {p}")
    if (p / "train.npy").exists():
        gt = np.load(p / "groundtruth.npy").astype(np.int64) if (p / "groundtruth.npy").exists() else None
        return np.load(p / "train.npy").astype(np.float32), np.load(p / "queries.npy").astype(np.float32), gt
    if (p / "base.fvecs").exists():
        gt = load_ivecs(p / "groundtruth.ivecs").astype(np.int64) if (p / "groundtruth.ivecs").exists() else None
        return load_fvecs(p / "base.fvecs"), load_fvecs(p / "query.fvecs"), gt
    raise ValueError(f"Could not detect dataset format in {p}. Expected train.npy+queries.npy or base.fvecs+query.fvecs.")


def timestamped_output_path(path: Path, now: Optional[datetime] = None) -> Path:
    """``name_YYYYMMDD_HHMMSS.suffix`` in UTC (reference :104-115)."""
    now = now or datetime.now(timezone.utc)
    return path.with_name(f"{path.stem}_{now.strftime('%Y%m%d_%H%M%S')}{path.suffix}")


def _pq_M(D: int, bpd: float) -> int:
    """Sub-quantizers at 8 bits each for a bpd budget, clamped to [1, D] (reference :142-146)."""
    return min(max(1, int(bpd * D) // 8), D)


def _sq_bits(bpd: float) -> int:
    """4 up to 4.5 bpd, 8 up to 12, else 16 (reference :157-163)."""
    return 4 if bpd <= 4.5 else 8 if bpd <= 12 else 16


def build_method_configs(method_names: list, D: int, bpd: float, K: int = 1024, nprobe: int = 64) -> dict:
    """method name -> unfitted ``BaseSearchIndex`` (reference :118-246)."""
    from haag_vq.methods.optimized_product_quantization import OptimizedProductQuantizer
    from haag_vq.methods.product_quantization import ProductQuantizer
    from haag_vq.methods.scalar_quantization import ScalarQuantizer
    from haag_vq.methods.search import FaissIvfPqIndex, FlatQuantizedIndex, RaBitQIndex

    configs = {}
    for name in method_names:
        if name == "pq_flat":
            configs[name] = FlatQuantizedIndex(ProductQuantizer(M=_pq_M(D, bpd), B=8))
        elif name == "sq_flat":
            configs[name] = FlatQuantizedIndex(ScalarQuantizer(num_bits=_sq_bits(bpd)))
        elif name == "faiss_ivfpq":
            configs[name] = FaissIvfPqIndex(K=K, m=_pq_M(D, bpd), nbits=8, nprobe=nprobe)
        elif name == "rabitq":  # ~1 bit per dimension by construction: bpd is ignored
            configs[name] = RaBitQIndex()
        elif name == "opq_flat":
            M = _pq_M(D, bpd)
            while M > 1 and D % M != 0:  # OPQ needs M | D
                M -= 1
            configs[name] = FlatQuantizedIndex(OptimizedProductQuantizer(M=M, B=8))
        elif name in NOT_IN_BUILD:
            print(f"WARNING: {name} unavailable (not part of the MI355X build, DESIGN.md §9)", file=sys.stderr)
        else:
            print(f"WARNING: unknown method '{name}' — skipped", file=sys.stderr)
    return configs


def parse_args(argv: Optional[list] = None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(description="VQ benchmark harness — compares BaseSearchIndex methods.",
                                 formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    ap.add_argument("--dataset", default="synthetic",
                    help="Dataset directory (train.npy+queries.npy or base.fvecs+query.fvecs), or 'synthetic'.")
    ap.add_argument("--methods", default="pq_flat,sq_flat,pq_ivf,faiss_ivfpq",
                    help="Comma-separated list of methods to benchmark.")
    ap.add_argument("--bpd", type=float, default=8.0, help="Bits per dimension.")
    ap.add_argument("--sweep-bpd", dest="sweep_bpd_values", type=str, default=None,
                    help="Comma-separated bpd values for a sweep of the single method given in --methods.")
    ap.add_argument("--k", type=int, default=10, help="Number of neighbors for recall and search.")
    ap.add_argument("--output", default=None, help="Path to save results CSV. Omit to skip saving.")
    ap.add_argument("--plot", action="store_true", help="Show (or save) Pareto plot after benchmarking.")
    ap.add_argument("--plot-save", default=None, help="File path to save the Pareto plot image (implies --plot).")
    ap.add_argument("--K", type=int, default=1024, help="Number of IVF centroids for IVF-based methods.")
    ap.add_argument("--nprobe", type=int, default=64, help="Number of IVF cells probed at search time.")
    return ap.parse_args(argv)


def main(argv: Optional[list] = None):
    """Runs the benchmark; returns the results DataFrame (the reference returns None)."""
    args = parse_args(argv)
    print(f"Loading dataset: {args.dataset!r} ...")
    X_train, X_query, gt = load_dataset(args.dataset)
    N, D = X_train.shape
    print(f"  X_train={X_train.shape}  X_query={X_query.shape}")
    if gt is None:
        print(f"  Computing brute-force ground truth (k={args.k}) ...")
        gt = compute_ground_truth(X_train, X_query, k=args.k)
    else:
        print(f"  Ground truth loaded: {gt.shape}")
    names = [m.strip() for m in args.methods.split(",") if m.strip()]

    if args.sweep_bpd_values is not None:
        if len(names) != 1:
            print("ERROR: --sweep-bpd requires exactly one method via --methods.", file=sys.stderr)
            sys.exit(1)
        values = [float(v) for v in args.sweep_bpd_values.split(",")]
        name = names[0]

        def factory(bpd: float):
            cfg = build_method_configs([name], D=D, bpd=bpd, K=args.K, nprobe=args.nprobe)
            if name not in cfg:
                raise RuntimeError(f"Could not instantiate method '{name}' — see warnings above.")
            return cfg[name]

        print(f"\nSweeping bpd={values} for method '{name}' ...")
        df = sweep_bpd(factory, values, X_train, X_query, gt, k=args.k)
    else:
        configs = build_method_configs(names, D=D, bpd=args.bpd, K=args.K, nprobe=args.nprobe)
        if not configs:
            print("ERROR: no methods could be instantiated.", file=sys.stderr)
            sys.exit(1)
        print(f"\nBenchmarking: {list(configs)} (k={args.k}, bpd={args.bpd})")
        df = compare_methods(configs, X_train, X_query, gt, k=args.k)

    print("\n--- Results ---")
    cols = [c for c in ("method", "bpd", "recall_at_k", "qps", "memory_bytes", "compression_ratio", "mse") if c in df.columns]
    print(df[cols].to_string(index=False))
    if args.output:
        out = timestamped_output_path(Path(args.output))
        out.parent.mkdir(parents=True, exist_ok=True)
        df.to_csv(out, index=False)
        print(f"\nSaved results to {out}")
    if args.plot or args.plot_save:
        pareto_plot(df, save_path=args.plot_save)
    return df


if __name__ == "__main__":
    main()
