"""Throughput of the other BASELINE.json configs on 1 GPU (bench.py measures the headline PQ16).

usage: python tools/bench_configs.py --workload opq32|sq8|rabitq1|ivfpq [--n N] [--steps K] [--warmup W]

  opq32   configs[2]: OPQ M=32 B=8 encode of 1M x 1536 (rotation on fp32 MFMA + PQ32 encode)
          and ADC recall@10 / queries/s (queries rotated, LUT + scan), OPQ trained on 65,536 rows.
  sq8     configs[3]: SQ-8 encode of 1M x 3072 (fit = per-dim min/max), and search by decode +
          exact scan (the reference's SQ search) for 100 queries.
  rabitq1 configs[3]: RaBitQ 1-bit encode of 1M x 3072, search by decode + exact scan, and the
          RaBitQIndex estimator search (qb 4) for --nq queries.
  ivfpq   SURVEY §8f rank 2: FaissIvfPqIndex defaults (K 4096, m 16, nbits 8, nprobe 200)
          over 1M x 1536: build (coarse k-means + residual PQ + add) time, search queries/s
          and recall@10 against exact ground truth.

Prints one JSON line in bench.py's format (roofline of the dominant kernel, HIP-event timing).
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))
from haag_vq import _native  # noqa: E402
from bench import synth, log  # noqa: E402

HBM_PEAK_GBS = 8000.0
MFMA_F32_PEAK_TFS = 157.3  # MI355X dense fp32 matrix (MI355X_MICROARCH.md chip table)


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for s, e in evs:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    dev_ms = float(np.mean([s.elapsed_time(e) for s, e in evs]))
    return wall, dev_ms


def recall(gt_ids, got_ids, k):
    return float(np.mean([len(set(gt_ids[j][:k]) & set(got_ids[j][:k])) / k for j in range(len(gt_ids))]))


def run_opq32(a, dev):
    from haag_vq.methods.optimized_product_quantization import OptimizedProductQuantizer

    d, M = 1536, 32
    X = synth(a.n, d, seed=0, dev=dev, kind="clustered")
    t0 = time.perf_counter()
    opq = OptimizedProductQuantizer(M=M, B=8)
    opq.niter = a.opq_iters
    opq.fit(X[:65536])
    torch.cuda.synchronize()
    log(f"OPQ fit on 65536 rows ({a.opq_iters} outer iterations): {time.perf_counter() - t0:.1f} s")
    A = opq.opq.A_device
    pq = opq.inner
    C = pq.centroids_device
    prep = _native.pq_prepare(C, 8)
    Y = torch.empty_like(X)
    codes = torch.empty((a.n, M), dtype=torch.uint8, device=dev)

    def rot():
        _native.opq_rotate(X, A, False, out=Y)

    def step():
        rot()
        _native.pq_encode(Y, C, prep, 8, out=codes)

    wall, dev_ms = timed(step, a.steps, a.warmup)
    _, rot_ms = timed(rot, a.steps, 1)
    Q = synth(a.nq, d, seed=1_000_003, dev=dev, kind="clustered")

    def search():
        lut = _native.adc_lut(_native.opq_rotate(Q, A, False), C, 8)
        return _native.adc_search(lut, codes, 10, 8)

    swall, sdev = timed(search, 3, 1)
    _, ai = search()
    _, gi = _native.flat_search(Q[:100].contiguous(), X, 10)
    rec = recall(gi.cpu().numpy(), ai[:100].cpu().numpy(), 10)
    flops = 2.0 * d * d * a.n
    return {
        "metric": "OPQ32 encode vectors/sec + ADC queries/sec @ recall@10, 1M×1536 fp32 (BASELINE configs[2])",
        "value": a.n / wall, "unit": "vectors/s", "ms_per_step": wall * 1e3, "dtype": "f32",
        "config": {"workload": f"opq32_encode_{a.n}x{d}", "M": M, "nbits": 8, "opq_outer_iters": a.opq_iters},
        "roofline": {"bound": "mfma", "kernel": "mivq_opq_rotate (rocBLAS fp32 sgemm)", "achieved": flops / (rot_ms * 1e-3) / 1e12,
                     "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s", "frac": flops / (rot_ms * 1e-3) / 1e12 / MFMA_F32_PEAK_TFS,
                     "rotate_ms": rot_ms, "encode_call_ms": dev_ms - rot_ms},
        "adc": {"qps": a.nq / swall, "nq": a.nq, "k": 10, "recall@10": rec, "recall_queries": 100,
                "ms_per_batch": swall * 1e3},
    }


def run_flatcodes(a, dev, kind):
    d = 3072
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    X = torch.randn((a.n, d), generator=g, device=dev, dtype=torch.float32)
    if kind == "sq8":
        lo = X.amin(0)
        hi = X.amax(0)
        den = (hi - lo) + 1e-8
        enc = lambda: _native.sq_encode(X, lo, den, 8)  # noqa: E731
        dec = lambda c: _native.sq_decode(c, d, lo, den, 8)  # noqa: E731
        bytes_per = 4 * d + d
    else:
        enc = lambda: _native.rabitq_encode(X, None, _native.METRIC_L2)  # noqa: E731
        dec = lambda c: _native.rabitq_decode(c, d, None)  # noqa: E731
        bytes_per = 4 * d + d // 8 + 8
    wall, dev_ms = timed(enc, a.steps, a.warmup)
    codes = enc()
    Q = X[:100].contiguous()  # reference convention: queries = first rows of the database

    def search():
        return _native.flat_search(Q, dec(codes), 10)

    swall, _ = timed(search, 2, 1)
    _, ai = search()
    _, gi = _native.flat_search(Q, X, 10)
    rec = recall(gi.cpu().numpy(), ai.cpu().numpy(), 10)
    ach = a.n * bytes_per / (dev_ms * 1e-3) / 1e9
    est = None
    if kind == "rabitq1":  # RaBitQIndex: IndexRaBitQ estimator search (center = mean, qb = 4)
        center = X.double().mean(0).float().contiguous()
        codes_c = _native.rabitq_encode(X, center, _native.METRIC_L2)
        Qe = X[: a.nq].contiguous()

        def est_search():
            return _native.rabitq_search(codes_c, d, center, Qe, 4, _native.METRIC_L2, 10)

        ewall, edev = timed(est_search, 3, 1)
        _, ei = est_search()
        est = {"qps": a.nq / ewall, "nq": a.nq, "k": 10, "qb": 4, "ms_per_batch": ewall * 1e3,
               "recall@10": recall(gi.cpu().numpy(), ei[:100].cpu().numpy(), 10),
               "codes_bytes": int(codes_c.numel()),
               "method": "mivq_rabitq_search: int8 MFMA over sign bits + estimator + tiled top-k"}
    return {
        "metric": f"{kind} encode vectors/sec + search queries/sec @ recall@10, 1M×3072 fp32 (BASELINE configs[3])",
        "value": a.n / wall, "unit": "vectors/s", "ms_per_step": wall * 1e3, "dtype": "f32",
        "config": {"workload": f"{kind}_encode_{a.n}x{d}"},
        "roofline": {"bound": "hbm", "kernel": f"{kind}_encode", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ach / HBM_PEAK_GBS, "bytes_per_vector": bytes_per, "kernel_ms": dev_ms},
        "search": {"qps": 100 / swall, "nq": 100, "k": 10, "recall@10": rec,
                   "method": "decode + exact L2 scan of the reconstructions (reference flat search)"},
        "estimator_search": est,
    }


def run_ivfpq(a, dev):
    from haag_vq.methods._ivf import IvfPq

    d, K, M = 1536, a.nlist, 16
    X = synth(a.n, d, seed=0, dev=dev, kind="clustered")
    idx = IvfPq(d, K, M, 8)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    idx.train(X)
    torch.cuda.synchronize()
    t_train = time.perf_counter() - t0
    t0 = time.perf_counter()
    idx.add(X)
    torch.cuda.synchronize()
    t_add = time.perf_counter() - t0
    Q = synth(a.nq, d, seed=1_000_003, dev=dev, kind="clustered")
    res = {}
    for nprobe in (a.nprobe, 16):
        swall, sdev = timed(lambda: idx.search(Q, 10, nprobe), a.steps, 1)
        _, ii = idx.search(Q[:100].contiguous(), 10, nprobe)
        _, gi = _native.flat_search(Q[:100].contiguous(), X, 10)
        res[nprobe] = {"qps": a.nq / swall, "ms_per_batch": swall * 1e3,
                       "recall@10": recall(gi.cpu().numpy(), ii.cpu().numpy(), 10)}
    # coarse-assignment kernel rate: one (rows x K x d) pairwise pass over 65,536 rows
    xs = X[:65536].contiguous()
    out = torch.empty((xs.shape[0], K), dtype=torch.float32, device=dev)
    _, pw_ms = timed(lambda: _native.pairwise_distances(xs, idx.coarse, _native.METRIC_L2, out=out), 5, 1)
    pair_steps = xs.shape[0] * K * d
    return {
        "metric": "IVF-PQ (K 4096, PQ16x8, nprobe 200) search queries/sec @ recall@10, 1M x 1536 fp32",
        "value": res[a.nprobe]["qps"], "unit": "queries/s", "ms_per_step": res[a.nprobe]["ms_per_batch"],
        "dtype": "f32", "config": {"workload": f"ivfpq_{a.n}x{d}", "nlist": K, "M": M, "nbits": 8,
                                    "nprobe": a.nprobe, "nq": a.nq, "k": 10},
        "search": res, "build_s": {"train": t_train, "add": t_add},
        "pairwise_kernel": {"ms": pw_ms, "rows": xs.shape[0], "cols": K, "d": d,
                            "pair_steps_per_s": pair_steps / (pw_ms * 1e-3),
                            "note": "sequential fmaf chains (sub + fma per pair-step) on packed fp32 VALU"},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=("opq32", "sq8", "rabitq1", "ivfpq"), required=True)
    ap.add_argument("--nlist", type=int, default=4096)
    ap.add_argument("--nprobe", type=int, default=200)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--opq-iters", type=int, default=10)
    a = ap.parse_args()
    dev = _native.require_device()
    if a.workload == "opq32":
        out = run_opq32(a, dev)
    elif a.workload == "ivfpq":
        out = run_ivfpq(a, dev)
    else:
        out = run_flatcodes(a, dev, a.workload)
    out.update({"n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "higher_is_better": True, "data": "synthetic"})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
