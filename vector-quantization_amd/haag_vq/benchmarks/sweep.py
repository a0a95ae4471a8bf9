"""`vq-benchmark sweep`: parameter sweeps over one quantizer family, one SQLite row per config.

The caller of the hot path named by the north star ("drops in behind `vq-benchmark sweep`",
BASELINE.json configs[0]).  Same options, grids, per-config pipeline and logged metrics as
/root/reference/src/haag_vq/benchmarks/sweep.py:
  * ``sweep`` (:48-219): codebooks dir (CLI > $CODEBOOKS_DIR > ./codebooks, created and not
    otherwise used, as upstream), optional precomputed ground truth (.npy), dataset, the
    grid of the method, then ``_run_single_config`` per config under one sweep id;
  * config generators (:221-319): PQ / OPQ = product of M and B lists, SQ keeps only 8-bit
    (others are skipped with a warning; 8-bit is the fallback), RaBitQ takes metric names
    or numbers of ``MetricType``;
  * ``_run_single_config`` (:390-517): fit, ``time_compress``, ``time_decompress``,
    distortion (per-vector SSE mean), compression ratio, pairwise distortion (seed 42),
    rank distortion, the ``measure_qps`` codebook-query proxy, recall@10/100, ``log_run``.
The quantizers, metrics and search run on the MI355X through libmivq (``haag_vq.methods``).

Deliberate differences: ``--db-path`` is forwarded to ``log_run`` (upstream drops it,
:196-207, so rows always went to $DB_PATH / logs/benchmark_runs.db); ``--method saq``
raises ValueError (upstream imports a removed module, :25-28; SAQ is out of scope here);
datasets that upstream downloads from the Hugging Face Hub are read from local files
(``$VQ_DATA_DIR/<name>.npy|.fvecs``, data/datasets.py) since there is no network.
"""

from __future__ import annotations

import itertools
import os
import uuid
from datetime import datetime
from pathlib import Path
from time import perf_counter
from typing import Any, Dict, List, Optional

import numpy as np
import typer

from haag_vq.data.datasets import Dataset, load_dummy_dataset, load_named_dataset
from haag_vq.methods.optimized_product_quantization import OptimizedProductQuantizer
from haag_vq.methods.product_quantization import ProductQuantizer
from haag_vq.methods.rabit_quantization import RaBitQuantizer
from haag_vq.methods.scalar_quantization import ScalarQuantizer
from haag_vq.metrics.distortion import compute_distortion
from haag_vq.metrics.pairwise_distortion import compute_pairwise_distortion
from haag_vq.metrics.performance import device_encode_roofline, measure_qps, time_compress, time_decompress
from haag_vq.metrics.rank_distortion import compute_rank_distortion
from haag_vq.metrics.recall import evaluate_recall
from haag_vq.utils.faiss_utils import MetricType
from haag_vq.parallel.launch import finish_rank, init_rank, launch_ranks, launched_world
from haag_vq.utils.run_logger import log_run

DATASETS = ("dummy", "huggingface", "cohere-msmarco", "dbpedia-100k", "dbpedia-1536", "dbpedia-3072")


def sweep(
    method: str = typer.Option("pq", help="Compression method: pq, sq, rabitq, opq, saq"),
    dataset: str = typer.Option(..., help="Dataset name (REQUIRED): " + ", ".join(DATASETS)),
    num_samples: int = typer.Option(10000, help="Number of samples to use (for dummy dataset)"),
    dim: int = typer.Option(1024, help="Dimensionality (for dummy dataset)"),
    dataset_limit: int = typer.Option(None, help="Limit number of vectors to load from dataset (None = load all available)"),
    cache_dir: str = typer.Option("../datasets", help="Directory of local dataset files (or $VQ_DATA_DIR)"),
    pq_subquantizers: str = typer.Option("8,16,32", help="[PQ only] Comma-separated subquantizer counts (M)"),
    pq_bits: str = typer.Option("8", help="[PQ only] Comma-separated bit values (B)"),
    sq_bits: str = typer.Option("8", help="[SQ only] Comma-separated bit values (e.g., '4,8,16')"),
    rabitq_metric_type: str = typer.Option("L2", help="[RabitQ only] Comma-separated metric distance types"),
    saq_num_bits: str = typer.Option("4,8", help="[SAQ only] out of scope in this build"),
    saq_total_bits: str = typer.Option("", help="[SAQ only] out of scope in this build"),
    saq_allowed_bits: str = typer.Option("0,2,4,6,8", help="[SAQ only] out of scope in this build"),
    saq_segments: str = typer.Option("", help="[SAQ only] out of scope in this build"),
    opq_quantizers: str = typer.Option("8,16,32", help="[OPQ only] Comma-separated number of quantizers"),
    opq_bits: str = typer.Option("8", help="[OPQ only] Comma-separated bit values"),
    with_recall: bool = typer.Option(True, help="Compute recall metrics"),
    with_pairwise: bool = typer.Option(True, help="Compute pairwise distance distortion"),
    with_rank: bool = typer.Option(True, help="Compute rank distortion"),
    num_pairs: int = typer.Option(1000, help="Number of random pairs for pairwise distortion"),
    rank_k: int = typer.Option(10, help="k for rank distortion (top-k neighbors)"),
    ground_truth_path: str = typer.Option(None, help="Path to precomputed ground truth (.npy file)"),
    codebooks_dir: str = typer.Option(None, help="Directory to save codebooks (default: ./codebooks or $CODEBOOKS_DIR)"),
    db_path: str = typer.Option(None, help="Path to SQLite database (default: logs/benchmark_runs.db or $DB_PATH)"),
    gpus: int = typer.Option(1, help="GPUs of this node: one process per GPU, the configurations dealt round-robin"),
    device: int = typer.Option(None, help="GPU index for a single-process sweep (default: the current device)"),
) -> str:
    """Run a parameter sweep and log every configuration to the run database.

    Examples:
        vq-benchmark sweep --method pq --dataset dummy --pq-subquantizers 8 --pq-bits 8
        vq-benchmark sweep --method sq --dataset dummy
    """
    if gpus > 1 and launched_world() == 1:
        # one process per GPU as a child command, before anything here touches the GPU
        sweep_id = f"sweep_{datetime.now().strftime('%Y%m%d_%H%M%S')}_{uuid.uuid4().hex[:8]}"
        args = ["sweep", "--method", method, "--dataset", dataset, "--num-samples", str(num_samples), "--dim", str(dim),
                "--cache-dir", cache_dir, "--pq-subquantizers", pq_subquantizers, "--pq-bits", pq_bits,
                "--sq-bits", sq_bits, "--rabitq-metric-type", rabitq_metric_type,
                "--opq-quantizers", opq_quantizers, "--opq-bits", opq_bits,
                "--num-pairs", str(num_pairs), "--rank-k", str(rank_k), "--gpus", str(gpus)]
        args += ["--with-recall" if with_recall else "--no-with-recall",
                 "--with-pairwise" if with_pairwise else "--no-with-pairwise",
                 "--with-rank" if with_rank else "--no-with-rank"]
        for flag, v in (("--dataset-limit", dataset_limit), ("--ground-truth-path", ground_truth_path),
                        ("--codebooks-dir", codebooks_dir), ("--db-path", db_path)):
            if v is not None:
                args += [flag, str(v)]
        rc = launch_ranks(gpus, args, extra_env={"VQ_SWEEP_ID": sweep_id})
        if rc != 0:
            raise RuntimeError(f"sweep: the {gpus}-rank run exited with {rc}")
        return sweep_id
    world = launched_world()
    if world > 1 and gpus != world:
        raise ValueError(f"sweep: --gpus {gpus} but WORLD_SIZE={world}")
    # configurations are dealt by RANK / WORLD_SIZE alone: no process group (no collective
    # to wait in while another rank runs a longer configuration)
    info = init_rank(device, collectives=False)

    if codebooks_dir is None:
        codebooks_dir = os.getenv("CODEBOOKS_DIR")
    codebooks_dir = Path(codebooks_dir) if codebooks_dir is not None else Path.cwd() / "codebooks"
    codebooks_dir.mkdir(parents=True, exist_ok=True)

    precomputed_gt = None
    if ground_truth_path:
        print(f"Loading precomputed ground truth from: {ground_truth_path}")
        precomputed_gt = np.load(ground_truth_path, allow_pickle=False)
        print(f"   Loaded ground truth shape: {precomputed_gt.shape}")

    sweep_id = os.environ.get("VQ_SWEEP_ID") or f"sweep_{datetime.now().strftime('%Y%m%d_%H%M%S')}_{uuid.uuid4().hex[:8]}"
    print("=" * 70)
    print("  HAAG Vector Quantization - Parameter Sweep (MI355X)")
    print("=" * 70)
    print(f"\nSweep ID: {sweep_id}")

    print(f"\nLoading dataset: {dataset}...")
    if dataset == "dummy":
        data = load_dummy_dataset(num_samples=num_samples, dim=dim)
    elif dataset in DATASETS:
        data = load_named_dataset(dataset, limit=dataset_limit, cache_dir=cache_dir)
    else:
        raise ValueError(f"Unsupported dataset: {dataset}. Supported: {', '.join(DATASETS)}")
    if precomputed_gt is not None:
        data.ground_truth = precomputed_gt
    print(f"Dataset shape: {data.vectors.shape}")

    if method == "pq":
        configs = _generate_pq_configs(pq_subquantizers, pq_bits)
    elif method == "sq":
        configs = _generate_sq_configs(sq_bits)
    elif method == "rabitq":
        configs = _generate_rabitq_configs(rabitq_metric_type)
    elif method == "opq":
        configs = _generate_opq_configs(opq_quantizers, opq_bits)
    elif method == "saq":
        raise ValueError("saq: the SAQ research method is out of scope of the MI355X build")
    else:
        raise ValueError(f"Unknown method: {method}. Supported: pq, sq, rabitq, opq, saq")

    print(f"\nRunning {len(configs)} configurations..." + (f" (rank {info.rank} of {info.world})" if info.world > 1 else ""))
    print("-" * 70)
    for i, config in enumerate(configs, 1):
        if (i - 1) % info.world != info.rank:  # --gpus N: configuration i runs on rank (i - 1) mod N
            continue
        print(f"\n[{i}/{len(configs)}] {config['name']}")
        _run_single_config(method=method, dataset=dataset, data=data, config=config, with_recall=with_recall,
                           with_pairwise=with_pairwise, with_rank=with_rank, num_pairs=num_pairs, rank_k=rank_k,
                           sweep_id=sweep_id, codebooks_dir=codebooks_dir, db_path=db_path, n_gpus=info.world)
    finish_rank(info)
    print("\n" + "=" * 70)
    print(f"  Sweep complete: {len(configs)} configurations, sweep id {sweep_id}")
    print(f"  Results logged to: {db_path or os.getenv('DB_PATH', 'logs/benchmark_runs.db')}")
    print("=" * 70)
    return sweep_id


def _ints(csv: str) -> List[int]:
    return [int(x.strip()) for x in csv.split(",")]


def _generate_pq_configs(subquantizers: str, bits: str) -> List[Dict[str, Any]]:
    """Product of the M and B lists (sweep.py:221-234)."""
    return [{"name": f"PQ(subquantizers={m}, bits={b})", "subquantizers": m, "bits": b}
            for m, b in itertools.product(_ints(subquantizers), _ints(bits))]


def _generate_sq_configs(bits: str) -> List[Dict[str, Any]]:
    """8-bit only, as upstream (sweep.py:237-263): other widths are skipped with a warning."""
    configs = []
    for num_bits in _ints(bits):
        if num_bits != 8:
            print(f"  Warning: SQ currently only supports 8-bit. Skipping {num_bits}-bit.")
            continue
        configs.append({"name": f"SQ({num_bits}-bit)", "num_bits": num_bits})
    return configs or [{"name": "SQ(8-bit)", "num_bits": 8}]


def _generate_rabitq_configs(metric_type: str) -> List[Dict[str, Any]]:
    """Metric names or numbers of MetricType, case-insensitive (sweep.py:266-303)."""
    out: List[Dict[str, Any]] = []
    for t in (t.strip() for t in metric_type.split(",") if t.strip()):
        parsed: Optional[MetricType] = None
        try:
            parsed = MetricType(int(t))
        except ValueError:
            parsed = next((m for m in MetricType if m.name.lower() == t.lower()), None)
        if parsed is None:
            raise ValueError(f"Unknown RabitQ metric type: '{t}'. Use numeric value or one of: "
                             + ", ".join(m.name for m in MetricType))
        out.append({"name": f"RabitQ(metric={parsed.name})", "metric_type": parsed})
    return out


def _generate_opq_configs(subquantizers: str, bits: str) -> List[Dict[str, Any]]:
    """Product of the M and B lists (sweep.py:305-318)."""
    return [{"name": f"OPQ(subquantizers={m}, bits={b})", "subquantizers": m, "bits": b}
            for m, b in itertools.product(_ints(subquantizers), _ints(bits))]


def _get_codebook_vectors(model: Any) -> Optional[np.ndarray]:
    """The (M*ksub, dsub) stacked PQ codebook, or SQ's [min; max] (sweep.py:367-387)."""
    if isinstance(model, ProductQuantizer):
        if not getattr(model, "codebooks", None):
            return None
        return np.concatenate([np.asarray(cb, dtype=np.float32) for cb in model.codebooks], axis=0)
    if isinstance(model, OptimizedProductQuantizer):
        if getattr(model, "pq", None) is None:
            return None
        return np.concatenate([np.asarray(cb, dtype=np.float32) for cb in model.inner.codebooks], axis=0)
    if isinstance(model, ScalarQuantizer):
        if model.min is None or model.max is None:
            return None
        return np.stack([model.min, model.max]).astype(np.float32)
    return None


def _build_model(method: str, config: Dict[str, Any]):
    if method == "pq":
        return ProductQuantizer(M=config["subquantizers"], B=config["bits"])
    if method == "sq":
        return ScalarQuantizer()  # always 8-bit, as upstream (sweep.py:411-413)
    if method == "rabitq":
        return RaBitQuantizer(metric_type=config["metric_type"])
    if method == "opq":
        return OptimizedProductQuantizer(M=config["subquantizers"], B=config["bits"])
    raise ValueError(f"Unsupported method: {method}")


def _run_single_config(method: str, dataset: str, data: Dataset, config: Dict[str, Any], with_recall: bool,
                       with_pairwise: bool, with_rank: bool, num_pairs: int, rank_k: int, sweep_id: str = None,
                       codebooks_dir: Path = None, db_path: str = None, n_gpus: int = 1) -> Dict[str, Any]:
    """Fit, encode, decode and score one configuration; log it; return its metrics.  Besides
    the reference's fields, metrics_json carries ``device``, ``n_gpus``, ``encode_device_ms`` and
    ``roofline_frac`` (the device encode of X against the 8 TB/s HBM roofline);
    config_json stays the reference's grid config."""
    model = _build_model(method, config)
    X = data.vectors
    t0 = perf_counter()
    model.fit(X)
    fit_time = perf_counter() - t0

    X_compressed, compression_time = time_compress(model, X)
    _, decompression_time = time_decompress(model, X_compressed)
    reconstruction_distortion = compute_distortion(X, X_compressed, model)
    compression_ratio = model.get_compression_ratio(X)
    metrics: Dict[str, Any] = {
        "reconstruction_distortion": reconstruction_distortion,
        "compression_ratio": compression_ratio,
        "fit_latency_ms": fit_time * 1000.0,
        "compression_latency_ms": compression_time * 1000.0,
        "decompression_latency_ms": decompression_time * 1000.0,
        "quantization_latency_ms": (fit_time + compression_time) * 1000.0,
    }
    pairwise = None
    if with_pairwise:
        pairwise = compute_pairwise_distortion(X, X_compressed, model, num_pairs=num_pairs)
        metrics["pairwise_distortion_mean"] = pairwise["mean"]
        metrics["pairwise_distortion_median"] = pairwise["median"]
        metrics["pairwise_distortion_max"] = pairwise["max"]
    rank_dist = None
    if with_rank:
        rank_dist = compute_rank_distortion(data, model, k=rank_k)
        metrics[f"rank_distortion@{rank_k}"] = rank_dist
    metrics.update(measure_qps(data.queries, model=model, codebook_vectors=_get_codebook_vectors(model)))
    if with_recall:
        metrics.update(evaluate_recall(data, model, num_queries=100))
    metrics.update(device_encode_roofline(model, X))
    metrics["n_gpus"] = int(n_gpus)

    log_run(method=method, dataset=dataset, metrics=metrics, config=config, sweep_id=sweep_id, db_path=db_path)

    print(f"  Compression ratio:           {compression_ratio:.2f}x")
    print(f"  Reconstruction MSE:          {reconstruction_distortion:.4f}")
    print(f"  Fit latency (ms):            {metrics['fit_latency_ms']:.2f}")
    print(f"  Compression latency (ms):    {metrics['compression_latency_ms']:.2f}")
    print(f"  Quantization latency (ms):   {metrics['quantization_latency_ms']:.2f}")
    print(f"  Decompression latency (ms):  {metrics['decompression_latency_ms']:.2f}")
    if pairwise is not None:
        print(f"  Pairwise distortion (mean):  {pairwise['mean']:.4f}")
    if rank_dist is not None:
        print(f"  Rank distortion@{rank_k}:       {rank_dist:.4f}")
    print(f"  QPS:                         {metrics['qps']:.2f}")
    if "recall@10" in metrics:
        print(f"  Recall@10:                  {metrics['recall@10']:.4f}")
    return metrics
