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

``--gpus N`` (BASELINE config #5's 53M x 1024 row-sharded encode): the command
starts N ranks (one process per GPU, parallel/launch.py) as a child; rank 0 trains the
quantizer and broadcasts it; the stream's batches (the first ``max_batches`` of them) are
dealt to the ranks in contiguous runs, so each rank reads and encodes its own rows with no
collective on the encode path; at the end one all-reduce collects the per-batch
(weighted distortion, count) pairs, which rank 0 sums in stream order -- the logged MSE is
the single-process value bit for bit -- and one all-reduce the ranks' encode times.
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
from haag_vq.parallel import sharded
from haag_vq.parallel.launch import comm_device, finish_rank, init_rank, launch_ranks, launched_world
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


def _batch_distortion(model, xb: torch.Tensor, codes) -> torch.Tensor:
    """compute_distortion (metrics/distortion.py:4-6) on the device-resident batch (a 0-d fp64
    device tensor: the caller collects them without a sync per batch)."""
    rec = model.decompress(codes)
    return ((xb.double() - rec.double()) ** 2).sum(1).mean()


# Stream batches per device encode call.  Upstream's loop calls compress once per 10,000-row
# batch (streaming_sweep.py:153-185); on the GPU a 10k-row call is launch- and prologue-bound
# (39 rows per filter workgroup), so consecutive batches of a rank's run go to the device
# together, ~2^20 rows per call (capped at 4 GiB of fp32 rows), and each batch's distortion is
# then computed from its own rows and codes exactly as before: codes are row-independent and
# the per-batch terms are the same tensors of the same shapes, so the logged row does not
# depend on the grouping (or on the number of ranks).
CALL_ROWS = 1 << 20
CALL_BYTES = 4 << 30


def batches_per_call(batch_size: int, dim: int) -> int:
    by_rows = max(1, CALL_ROWS // max(1, batch_size))
    by_bytes = max(1, CALL_BYTES // max(1, batch_size * dim * 4))
    return min(by_rows, by_bytes)


def batch_plan(n_total: int, batch_size: int, max_batches: Optional[int], rank: int = 0,
               world: int = 1) -> tuple:
    """(first rows of all batches of the run, this rank's batch index range [b0, b1)): the
    stream's batches in order, truncated to ``max_batches``, in contiguous runs per rank."""
    starts = list(range(0, n_total, batch_size))
    if max_batches:
        starts = starts[:max_batches]
    return starts, sharded.shard_range(len(starts), rank, world)


def _dry_run(stream, batch_size, max_batches, info, sweep_id, say) -> str:
    """--dry-run: the launcher, batch plan and the final reduction over gloo on the host; each
    batch contributes (sum of squares, rows).  Rank 0 prints one JSON line with the totals."""
    import json

    n_total = stream.shape[0]
    starts, (b0, b1) = batch_plan(n_total, batch_size, max_batches, info.rank, info.world)
    part = np.zeros((len(starts), 2), dtype=np.float64)
    for b in range(b0, b1):
        xb = np.asarray(stream[starts[b]:starts[b] + batch_size], dtype=np.float64)
        part[b] = (float((xb * xb).sum()), xb.shape[0])
    if info.world > 1:
        t = torch.from_numpy(part)
        torch.distributed.all_reduce(t)
        part = t.numpy()
    tot = 0.0
    for v, _ in part:
        tot += float(v)
    if info.rank == 0:
        say(json.dumps({"dry_run": True, "sweep_id": sweep_id, "world": info.world, "batches": len(starts),
                        "rows": int(part[:, 1].sum()), "sum_sq": tot}))
    finish_rank(info)
    return sweep_id


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
    gpus: int = typer.Option(1, help="GPUs of this node: the stream's batches row-sharded, one process per GPU"),
    dry_run: bool = typer.Option(False, "--dry-run", hidden=True,
                                 help="CPU rehearsal of the rank plumbing: no quantizer; each batch's value is its "
                                      "sum of squares"),
) -> str:
    """Train on a subset, then stream-compress the whole dataset in batches (one logged row)."""
    path = _resolve_path(dataset, data_path, cache_dir)
    if gpus > 1 and launched_world() == 1:
        # one process per GPU as a child command, before anything here touches the GPU
        sweep_id = f"streaming_{method}_{datetime.now().strftime('%Y%m%d_%H%M%S')}_{uuid.uuid4().hex[:8]}"
        args = ["streaming-sweep", "--method", method, "--dataset", dataset, "--training-size", str(training_size),
                "--batch-size", str(batch_size), "--cache-dir", cache_dir, "--data-path", str(path),
                "--pq-subquantizers", pq_subquantizers, "--pq-bits", pq_bits, "--opq-quantizers", opq_quantizers,
                "--opq-bits", opq_bits, "--gpus", str(gpus)] + (["--dry-run"] if dry_run else [])
        if max_batches:
            args += ["--max-batches", str(max_batches)]
        if db_path:
            args += ["--db-path", db_path]
        rc = launch_ranks(gpus, args, extra_env={"VQ_SWEEP_ID": sweep_id})
        if rc != 0:
            raise RuntimeError(f"streaming-sweep: the {gpus}-rank run exited with {rc}")
        return sweep_id
    world = launched_world()
    if world > 1 and gpus != world:
        raise ValueError(f"streaming-sweep: --gpus {gpus} but WORLD_SIZE={world}")
    info = init_rank()
    head = info.rank == 0
    stream = open_vector_stream(path)
    sweep_id = os.environ.get("VQ_SWEEP_ID") or \
        f"streaming_{method}_{datetime.now().strftime('%Y%m%d_%H%M%S')}_{uuid.uuid4().hex[:8]}"
    n_total, dim = stream.shape
    say = print if head else (lambda *a, **k: None)
    say("=" * 70)
    say("  Streaming Batch Compression (MI355X)")
    say("=" * 70)
    say(f"Sweep ID: {sweep_id}\nMethod: {method}\nVectors: {n_total:,} x {dim}\n"
        f"Training size: {training_size:,}\nBatch size: {batch_size:,}\nGPUs: {info.world}")

    training = np.ascontiguousarray(stream[:training_size], dtype=np.float32) if head else \
        np.empty((0, dim), np.float32)
    if dry_run:
        return _dry_run(stream, batch_size, max_batches, info, sweep_id, say)
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
    say(f"\n[1/3] Training {method} quantizer on {len(training):,} vectors...")
    if head:
        model.fit(training)
    model = sharded.broadcast_quantizer(model if head else None)

    say("\n[2/3] Streaming and compressing in batches...")
    starts, (b0, b1) = batch_plan(n_total, batch_size, max_batches, info.rank, info.world)
    part = np.zeros((len(starts), 2), dtype=np.float64)  # per batch: mse * count, count
    timers = []
    per_call = batches_per_call(batch_size, dim)
    mse_dev = []  # (batch index, 0-d fp64 device tensor)
    for g0 in range(b0, b1, per_call):
        g1 = min(b1, g0 + per_call)
        r0, r1 = starts[g0], min(n_total, starts[g1 - 1] + batch_size)
        xg = _arrays.to_device(np.ascontiguousarray(stream[r0:r1], dtype=np.float32))
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        codes = model.compress(xg)  # one device call for the batches g0 .. g1-1
        ev[1].record()
        timers.append(ev)
        for b in range(g0, g1):
            s, e = starts[b] - r0, min(n_total, starts[b] + batch_size) - r0
            # the batch's codes as a fresh allocation, as a per-batch call returned them
            mse_dev.append((b, _batch_distortion(model, xg[s:e], codes[s:e].clone())))
            part[b, 1] = e - s
            if head and (b - b0 + 1) % 100 == 0:
                say(f"  Compressed {b - b0 + 1} batches on rank 0 ({int(part[b0:b + 1, 1].sum()):,} vectors)")
        del xg, codes
    torch.cuda.synchronize()
    if mse_dev:
        vals = torch.stack([t for _, t in mse_dev]).cpu().numpy()
        for (b, _), v in zip(mse_dev, vals):
            part[b, 0] = float(v) * part[b, 1]  # weighted, as upstream
    enc_s = sum(e0.elapsed_time(e1) for e0, e1 in timers) * 1e-3
    ratio = model.get_compression_ratio(training)
    code_bytes = 4 * dim / ratio  # bytes per encoded vector (every ratio is 4 D / code bytes)
    if info.world > 1:  # one all-reduce each: batch values (every batch on one rank), the encode times
        cdev = comm_device(info)
        t = torch.from_numpy(part).to(cdev)
        torch.distributed.all_reduce(t)
        part = t.cpu().numpy()
        tm = torch.tensor([enc_s], dtype=torch.float64, device=cdev)
        torch.distributed.all_reduce(tm, op=torch.distributed.ReduceOp.MAX)
        enc_s = float(tm.cpu())
    if max_batches and len(starts) >= max_batches:
        say(f"  Reached max batches limit ({max_batches})")

    mse_sum = 0.0
    for v, _ in part:  # stream order, as the single-process loop adds them
        mse_sum += float(v)
    total, batches = int(part[:, 1].sum()), len(starts)
    say("\n[3/3] Finalizing metrics...")
    metrics = {"compression_ratio": ratio,
               "mse": mse_sum / total if total else 0.0,
               "total_vectors_compressed": total, "num_batches": batches,
               "n_gpus": info.world,
               "device": torch.cuda.get_device_name(info.device) if info.device is not None else None,
               "encode_device_s": enc_s,
               "encode_vectors_per_s": total / enc_s if enc_s > 0 else None,
               # bytes of the encode (fp32 rows read + codes written) / slowest rank's encode
               # time / (8 TB/s x GPUs): the fraction of the node's HBM roofline
               "roofline_frac": (total * (4 * dim + code_bytes) / enc_s / (8.0e12 * info.world)
                                 if enc_s > 0 else None)}
    if head:
        log_run(method=method, dataset=f"{dataset}-streaming", metrics=metrics, config=config, sweep_id=sweep_id,
                db_path=db_path)
    say(f"  Compression ratio: {metrics['compression_ratio']:.1f}x\n  MSE: {metrics['mse']:.6f}\n"
        f"  Total vectors: {total:,}")
    finish_rank(info)
    return sweep_id
