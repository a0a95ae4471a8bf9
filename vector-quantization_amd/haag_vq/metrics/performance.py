"""Latency / QPS metrics — /root/reference/src/haag_vq/metrics/performance.py:19-89.

Timers synchronise the HIP device before reading the clock so a measurement covers the
kernels it launched (the reference's CPU calls are synchronous).
"""

from time import perf_counter
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from haag_vq.methods.base_quantizer import BaseQuantizer
from haag_vq.methods.rabit_quantization import RaBitQuantizer
from haag_vq.utils.faiss_export import query_codebook


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def time_compress(model: BaseQuantizer, X) -> Tuple[np.ndarray, float]:
    _sync()
    t0 = perf_counter()
    codes = model.compress(X)
    _sync()
    return codes, float(perf_counter() - t0)


def time_decompress(model: BaseQuantizer, codes) -> Tuple[np.ndarray, float]:
    _sync()
    t0 = perf_counter()
    rec = model.decompress(codes)
    _sync()
    return rec, float(perf_counter() - t0)


HBM_PEAK_BYTES_PER_S = 8.0e12  # MI355X HBM3E


def device_encode_roofline(model: BaseQuantizer, X, reps: int = 3) -> Dict[str, object]:
    """Device time of ``model.compress`` on device-resident rows (HIP events, best of ``reps``
    after one warm-up) and its fraction of the HBM roofline: (bytes of X read + code bytes
    written) / time / 8 TB/s.  Logged next to the reference's host-timed latencies
    (the ``device`` / ``n_gpus`` / ``roofline_frac`` fields)."""
    if not torch.cuda.is_available():
        return {}
    Xd = X if isinstance(X, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(X))
    Xd = Xd.to(torch.cuda.current_device())
    codes = model.compress(Xd)
    best = float("inf")
    for _ in range(max(1, reps)):
        s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s_.record()
        codes = model.compress(Xd)
        e_.record()
        e_.synchronize()
        best = min(best, s_.elapsed_time(e_) * 1e-3)
    cb = codes.numel() * codes.element_size() if isinstance(codes, torch.Tensor) else int(np.asarray(codes).nbytes)
    nbytes = Xd.numel() * Xd.element_size() + cb
    return {"device": torch.cuda.get_device_name(torch.cuda.current_device()),
            "encode_device_ms": best * 1e3,
            "roofline_frac": nbytes / best / HBM_PEAK_BYTES_PER_S if best > 0 else None}


def measure_qps(queries, *, model: Optional[BaseQuantizer] = None, codebook_vectors: Optional[np.ndarray] = None,
                codebook_path: Optional[str] = None, repeats: int = 3, topk: int = 1) -> Dict[str, float]:
    """Reference "QPS" proxy: codebook query (PQ-like / SQ) or compress(queries) (RaBitQ)."""
    queries = np.asarray(queries, dtype=np.float32)
    if queries.ndim == 1:
        queries = queries.reshape(1, -1)
    if queries.size == 0:
        raise ValueError("No queries provided for QPS measurement")
    runs = max(1, repeats)
    if isinstance(model, RaBitQuantizer):
        def once():
            model.compress(queries)
    else:
        def once():
            query_codebook(queries, model=model, codebook_vectors=codebook_vectors, codebook_path=codebook_path,
                           topk=topk)
    durations: List[float] = []
    for _ in range(runs):
        _sync()
        t0 = perf_counter()
        once()
        _sync()
        durations.append(max(perf_counter() - t0, 1e-12))
    nq = float(len(queries))
    qps = [nq / d for d in durations]
    lat = [d / nq * 1000.0 for d in durations]
    return {"qps": float(np.mean(qps)), "qps_std": float(np.std(qps, ddof=0)),
            "avg_query_latency_ms": float(np.mean(lat)), "latency_ms_std": float(np.std(lat, ddof=0))}
