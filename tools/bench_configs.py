"""Throughput of the other BASELINE.json configs on 1 GPU, one at a time (bench.py runs the
opq32 / sq8 / rabitq1 legs itself as its `configs` key; ivfpq lives only here).

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
from bench import synth, log, opq32_leg, flatcodes_leg  # noqa: E402

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
    ap.add_argument("--data", choices=("gaussian", "clustered"), default="clustered")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work (bench.py's option)")
    a = ap.parse_args()
    dev = _native.require_device()
    if a.workload == "opq32":
        out = opq32_leg(a, dev, a.steps, a.warmup)
    elif a.workload == "ivfpq":
        out = run_ivfpq(a, dev)
    else:
        out = flatcodes_leg(a, dev, a.workload, a.steps, a.warmup)
    out.update({"n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "higher_is_better": True, "data": "synthetic"})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
