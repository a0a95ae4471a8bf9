"""`vq-benchmark streaming-sweep`: train on a subset, encode the whole set in batches.

Same pipeline as /root/reference/src/haag_vq/benchmarks/streaming_sweep.py:41-228 (the
53M x 1024 MS MARCO encode of BASELINE.json configs[4]): fit the quantizer on the first
``training_size`` vectors (:84-128), then compress the stream batch by batch and keep the
batch-size-weighted mean of the per-batch distortion (:153-185), then log one row with
dataset ``<name>-streaming`` (:208-214).

Upstream streams the Cohere embeddings from the Hugging Face Hub; offline, the stream is a
local file read through a memory map (``--data-path`` or ``$VQ_DATA_DIR/<dataset>.npy``;
``.fvecs`` too), so only one batch is in host memory at a time.  Each batch goes to the
device once: it is encoded there (``mivq_pq_encode`` / SQ / RaBitQ kernels) and its
distortion is computed from the device-resident batch and codes.
"""

from __future__ import annotations

import os
import uuid
from datetime import datetime
from pathlib import Path
from typing import Optional

import numpy as np
import torch
import typer

from haag_vq import _arrays
from haag_vq.methods.optimized_product_quantization import OptimizedProductQuantizer
from haag_vq.methods.product_quantization import ProductQuantizer
from haag_vq.methods.rabit_quantization import RaBitQuantizer
from haag_vq.methods.scalar_quantization import ScalarQuantizer
from haag_vq.utils.faiss_utils import MetricType
from haag_vq.utils.run_logger import log_run


def open_vector_stream(path) -> np.ndarray:
    """(N, D) float32 view of a .npy (memory-mapped) or .fvecs (strided memmap) file."""
    path = Path(path)
    if path.suffix == ".npy":
        return np.load(path, mmap_mode="r", allow_pickle=False)
    if path.suffix == ".fvecs":
        head = np.fromfile(path, dtype=np.int32, count=1)
        if head.size == 0:
            return np.empty((0, 0), np.float32)
        d = int(head[0])
        raw = np.memmap(path, dtype=np.float32, mode="r")
        if raw.size % (d + 1):
            raise ValueError(f"Corrupt vector file: {path}")
        return raw.reshape(-1, d + 1)[:, 1:]
    raise ValueError(f"unsupported vector file {path} (use .npy or .fvecs)")


def _resolve_path(dataset: str, data_path: Optional[str], cache_dir: str) -> Path:
    if data_path:
        return Path(data_path)
    root = Path(os.environ.get("VQ_DATA_DIR", cache_dir))
    for ext in (".npy", ".fvecs"):
        if (root / f"{dataset}{ext}").exists():
            return root / f"{dataset}{ext}"
    raise FileNotFoundError(f"{dataset}: upstream streams it from the Hugging Face Hub; offline, pass --data-path "
                            f"or place {dataset}.npy / .fvecs under {root} (or set VQ_DATA_DIR)")


def _batch_distortion(model, xb: torch.Tensor, codes) -> float:
    """compute_distortion (metrics/distortion.py:4-6) on the device-resident batch."""
    rec = model.decompress(codes)
    return float(((xb.double() - rec.double()) ** 2).sum(1).mean())


def streaming_sweep(
    method: str = typer.Option("pq", help="Compression method: pq, opq, sq, saq, rabitq"),
    dataset: str = typer.Option("cohere-msmarco", help="Dataset name (a local file, see --data-path)"),
    training_size: int = typer.Option(1_000_000, help="Number of vectors to use for training quantizer"),
    batch_size: int = typer.Option(10_000, help="Batch size for streaming compression"),
    max_batches: Optional[int] = typer.Option(None, help="Max batches to compress (None = all)"),
    cache_dir: str = typer.Option("../datasets", help="Directory of local dataset files (or $VQ_DATA_DIR)"),
    data_path: Optional[str] = typer.Option(None, help="Local .npy / .fvecs file to stream"),
    pq_subquantizers: str = typer.Option("16", help="[PQ] M value"),
    pq_bits: str = typer.Option("8", help="[PQ] B value"),
    opq_quantizers: str = typer.Option("16", help="[OPQ] M value"),
    opq_bits: str = typer.Option("8", help="[OPQ] B value"),
    saq_num_bits: str = typer.Option("4", help="[SAQ] out of scope in this build"),
    db_path: str = typer.Option(None, help="SQLite database path"),
) -> str:
    """Train on a subset, then stream-compress the whole dataset in batches (one logged row)."""
    stream = open_vector_stream(_resolve_path(dataset, data_path, cache_dir))
    sweep_id = f"streaming_{method}_{datetime.now().strftime('%Y%m%d_%H%M%S')}_{uuid.uuid4().hex[:8]}"
    n_total, dim = stream.shape
    print("=" * 70)
    print("  Streaming Batch Compression (MI355X)")
    print("=" * 70)
    print(f"Sweep ID: {sweep_id}\nMethod: {method}\nVectors: {n_total:,} x {dim}\n"
          f"Training size: {training_size:,}\nBatch size: {batch_size:,}")

    training = np.ascontiguousarray(stream[:training_size], dtype=np.float32)
    if method == "pq":
        M, B = int(pq_subquantizers), int(pq_bits)
        model, config = ProductQuantizer(M=M, B=B), {"M": M, "B": B}
    elif method == "opq":
        M, B = int(opq_quantizers), int(opq_bits)
        model, config = OptimizedProductQuantizer(M=M, B=B), {"M": M, "B": B}
    elif method == "sq":
        model, config = ScalarQuantizer(), {}
    elif method == "rabitq":
        model, config = RaBitQuantizer(metric_type=MetricType.L2), {}
    elif method == "saq":
        raise ValueError("saq: the SAQ research method is out of scope of the MI355X build")
    else:
        raise ValueError(f"Unknown method: {method}")
    print(f"\n[1/3] Training {method} quantizer on {len(training):,} vectors...")
    model.fit(training)

    print("\n[2/3] Streaming and compressing in batches...")
    total, batches, mse_sum = 0, 0, 0.0
    for s in range(0, n_total, batch_size):
        xb = _arrays.to_device(np.ascontiguousarray(stream[s:s + batch_size], dtype=np.float32))
        codes = model.compress(xb)
        mse_sum += _batch_distortion(model, xb, codes) * xb.shape[0]  # weighted, as upstream
        total += xb.shape[0]
        batches += 1
        if batches % 100 == 0:
            print(f"  Compressed {batches} batches ({total:,} vectors)")
        if max_batches and batches >= max_batches:
            print(f"  Reached max batches limit ({max_batches})")
            break

    print("\n[3/3] Finalizing metrics...")
    metrics = {"compression_ratio": model.get_compression_ratio(training),
               "mse": mse_sum / total if total else 0.0,
               "total_vectors_compressed": total, "num_batches": batches}
    log_run(method=method, dataset=f"{dataset}-streaming", metrics=metrics, config=config, sweep_id=sweep_id,
            db_path=db_path)
    print(f"  Compression ratio: {metrics['compression_ratio']:.1f}x\n  MSE: {metrics['mse']:.6f}\n"
          f"  Total vectors: {total:,}")
    return sweep_id
