"""Benchmark: PQ-encode vectors/s (+ ADC queries/s @ recall@10) on synthetic N x 1536 fp32.

Workload (BASELINE.json configs[1]): PQ M=16 B=8 encode of 1M x 1536 fp32 per GPU
(weak scaling: every rank owns its own 1M-row shard, generated on its device from seed =
rank, unit-normalised rows).  One "step" = one encode pass over the resident shard through
libmivq (mivq_pq_encode: fp16-MFMA filter kernel, exact resolve kernel, code transpose).
Codebooks: rank 0 trains them on its first 65,536 rows (GPU k-means, 25 iterations,
seed 1234) and broadcasts them (RCCL).  After the timed encode, the ADC leg searches the
encoded shards for `--nq` queries (broadcast from rank 0; per-shard top-10, RCCL
all-gather, on-device merge) and reports queries/s and recall@10 against the exact top-10
over the raw vectors.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        (N > 1: launched by torch.distributed.run, one rank per GPU)
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))

from haag_vq import _native  # noqa: E402
from haag_vq.methods._kmeans import train_pq  # noqa: E402
from haag_vq.parallel import sharded  # noqa: E402

METRIC = "PQ-encode vectors/sec + ADC queries/sec @ recall@10, 1M×1536 fp32"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=1_000_000, help="rows per GPU")
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--nq", type=int, default=1000, help="ADC queries")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--gt-queries", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-adc", action="store_true")
    ap.add_argument("--exact", action="store_true", help="force the exact VALU encode path")
    ap.add_argument("--legacy", action="store_true", help="diagnostic: subspace-looping MFMA kernel")
    ap.add_argument("--data", choices=("clustered", "gaussian"), default="clustered")
    ap.add_argument("--no-alt-data", action="store_true",
                    help="skip the second encode measurement on the other synthetic distribution")
    return ap.parse_args()


def synth(n, d, seed, dev, kind="clustered", centers_seed=12345, n_centers=4096, spread=0.02):
    """Synthetic embedding-like rows, generated on the device.

    gaussian : isotropic N(0, I) rows, L2-normalised (no neighbourhood structure: recall@k of
               any quantizer is ~0 on it, and it is the worst case for the encode filter).
    clustered: normalise(center[j] + spread * N(0, I)) with 4096 shared unit centers (seeded
               identically on every rank) — neighbourhoods like real text embeddings.
    """
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    if kind == "gaussian":
        X = torch.randn((n, d), generator=g, device=dev, dtype=torch.float32)
    else:
        gc = torch.Generator(device=dev)
        gc.manual_seed(centers_seed)
        cen = torch.randn((n_centers, d), generator=gc, device=dev, dtype=torch.float32)
        cen /= torch.linalg.vector_norm(cen, dim=1, keepdim=True)
        X = torch.empty((n, d), device=dev, dtype=torch.float32)
        step = 1 << 18
        for s in range(0, n, step):
            e = min(n, s + step)
            a = torch.randint(0, n_centers, (e - s,), generator=g, device=dev)
            X[s:e] = cen[a] + spread * torch.randn((e - s, d), generator=g, device=dev, dtype=torch.float32)
    X /= torch.linalg.vector_norm(X, dim=1, keepdim=True)
    return X.contiguous()


def traffic_from_profile(workload: str):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary, if it is for this workload."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None
    try:
        t = json.loads(p.read_text())
        return t.get(workload, {}).get("bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(X: torch.Tensor, C: np.ndarray, codes_dev: torch.Tensor, target_s: float):
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O  # CPU restatement: the baseline leg and the live parity check

    threads = O.cpu_threads()
    n_cal = 2000
    Xc = X[:n_cal].cpu().numpy()
    t0 = time.perf_counter()
    O.pq_encode(Xc, C)
    dt = time.perf_counter() - t0
    n_s = int(min(X.shape[0], max(n_cal, n_cal * target_s / max(dt, 1e-6))))
    Xs = X[:n_s].cpu().numpy()
    t0 = time.perf_counter()
    ref = O.pq_encode(Xs, C)
    dt = time.perf_counter() - t0
    got = codes_dev[:n_s].cpu().numpy()
    mism = int((got != ref).sum())
    return {
        "value": n_s / dt,
        "unit": "vectors/s",
        "cores": threads,
        "kind": "port",
        "sample": f"first {n_s} rows of rank 0's shard, oracle/mivq_oracle.c pq_encode (OpenMP, AVX2), {dt:.1f} s wall on {threads} threads = {dt * threads:.0f} thread-s",
    }, {"rows_checked": n_s, "mismatched_codes": mism}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = _native.require_device()
    nbits = 8
    log(f"[rank {rank}] generating {a.n}x{a.d} on {torch.cuda.get_device_name(dev)}")
    X = synth(a.n, a.d, seed=rank, dev=dev, kind=a.data)

    # codebooks: rank 0 trains, everyone receives (replicated, §8e)
    C = torch.empty((a.M, 256, a.d // a.M), dtype=torch.float32, device=dev)
    if rank == 0:
        t0 = time.perf_counter()
        C.copy_(train_pq(X[:65536], a.M, nbits, niter=25, seed=1234, exact_assign=True))
        torch.cuda.synchronize()
        log(f"[rank 0] k-means fit on 65536 rows: {time.perf_counter() - t0:.2f} s")
    if world > 1:
        dist.broadcast(C, src=0)
    prep = _native.pq_prepare(C, nbits)
    codes = torch.empty((a.n, _native.pq_code_size(a.M, nbits)), dtype=torch.uint8, device=dev)

    def step():
        _native.pq_encode(X, C, prep, nbits, exact=a.exact, out=codes,
                          flags_extra=_native.MIVQ_PQ_LEGACY_MFMA if a.legacy else 0)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for s, e in evs:
        s.record()
        step()
        e.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in evs]))
    value = world * a.n * a.steps / dt
    log(f"[rank {rank}] encode: {dt / a.steps * 1e3:.3f} ms/step wall, {kern_ms:.3f} ms/step device")

    bytes_per_vec = 4 * a.d + a.M  # read x, write codes
    achieved = a.n * bytes_per_vec / (kern_ms * 1e-3) / 1e9
    workload = f"pq{a.M}_encode_{a.n}x{a.d}"

    alt = None
    if rank == 0 and world == 1 and not a.no_alt_data:
        # the same encode on the other synthetic distribution (SURVEY §8d names unit-normalised
        # Gaussian rows; the headline uses clustered, embedding-like rows): own codebooks, same
        # step count, checked against the oracle on its first 20,000 rows
        kind = "gaussian" if a.data == "clustered" else "clustered"
        Xa = synth(a.n, a.d, seed=rank + 7, dev=dev, kind=kind)
        Ca = train_pq(Xa[:65536], a.M, nbits, niter=25, seed=1234, exact_assign=True).contiguous()
        prep_a = _native.pq_prepare(Ca, nbits)
        codes_a = torch.empty_like(codes)
        fa = lambda: _native.pq_encode(Xa, Ca, prep_a, nbits, out=codes_a)  # noqa: E731
        for _ in range(a.warmup):
            fa()
        torch.cuda.synchronize()
        ev_a = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
        t0 = time.perf_counter()
        for s_, e_ in ev_a:
            s_.record()
            fa()
            e_.record()
        torch.cuda.synchronize()
        dta = (time.perf_counter() - t0) / a.steps
        ms_a = float(np.mean([s_.elapsed_time(e_) for s_, e_ in ev_a]))
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle as O  # parity check of the alternate run (test infrastructure)
        ns = min(a.n, 20000)
        mism = int((codes_a[:ns].cpu().numpy() != O.pq_encode(Xa[:ns].cpu().numpy(), Ca.cpu().numpy())).sum())
        ach_a = a.n * (4 * a.d + a.M) / (ms_a * 1e-3) / 1e9
        alt = {"data": kind, "value": a.n / dta, "unit": "vectors/s", "ms_per_step": dta * 1e3, "kernel_ms": ms_a,
               "roofline_frac": ach_a / HBM_PEAK_GBS, "parity": {"rows_checked": ns, "mismatched_codes": mism}}
        log(f"[rank 0] alt data: {alt}")
        del Xa, codes_a

    adc = None
    if not a.no_adc:
        Q = synth(a.nq, a.d, seed=1_000_003, dev=dev, kind=a.data)
        adc = sharded.bench_adc(X, C, codes, nbits, rank, world, dev, Q, k=a.k, gt_queries=a.gt_queries)
        if rank == 0:
            log(f"[rank 0] adc: {adc}")

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu, parity = cpu_baseline(X, C.cpu().numpy(), codes, a.cpu_seconds)
        log(f"[rank 0] cpu baseline: {cpu}; parity {parity}")

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "vectors/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic {a.data} (see synth(): generated on device, seed = rank, rows L2-normalised); "
                    "codebooks from GPU k-means on the first 65,536 rows (seed 1234, 25 iterations)",
            "config": {"workload": workload, "rows_per_gpu": a.n, "dim": a.d, "M": a.M, "nbits": nbits,
                       "path": "exact" if a.exact else ("legacy-mfma" if a.legacy else "cs-mfma-filter+exact-recheck"),
                       "data": a.data,
                       "parallelism": f"row-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic_from_profile(workload),
                         "kernel": "mivq_pq_encode call: pq_encode_cs_kernel (filter) + pq_resolve_full2_kernel and "
                                   "pq_resolve_cs_kernel (exact re-check of the row-subspaces the filter could not "
                                   "settle) + pq_transpose_codes16_kernel",
                         "bytes_per_vector": bytes_per_vec, "kernel_ms": kern_ms},
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "adc": adc,
            "alt_data": alt,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
