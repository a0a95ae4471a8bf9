"""Interleaved A/B of mivq_rabitq_search (RaBitQ estimator search, qb = 4) between this build and
another libmivq.so: same codes and queries, ids and keys compared bit for bit, median per-call
time of alternating calls (HIP events).

usage: python tools/probe_rq.py OTHER.so|none [--n 1000000] [--d 3072] [--nq 1000] [--k 10] [--reps 5]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT / "tools"))
from haag_vq import _native  # noqa: E402
from ab_lib import bind  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("other")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=3072)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--qb", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = _native.require_device()
    g = torch.Generator(device=dev).manual_seed(2)
    codes = torch.empty((a.n, _native.rabitq_code_size(a.d)), dtype=torch.uint8, device=dev)
    for s in range(0, a.n, 200_000):  # encode in slices: 200k x 3072 fp32 at a time
        X = torch.randn((min(200_000, a.n - s), a.d), generator=g, device=dev)
        codes[s:s + X.shape[0]] = _native.rabitq_encode(X, None, _native.METRIC_L2)
    Q = torch.randn((a.nq, a.d), generator=g, device=dev)
    libs = {"this": bind(_native.LIB_PATH)}
    if a.other != "none":  # "none": this build alone (PMC passes)
        libs["other"] = bind(a.other if Path(a.other).is_absolute() else ROOT / a.other)
    st = torch.cuda.current_stream().cuda_stream
    P = ctypes.c_void_p
    out = {}
    for name, lb in libs.items():
        ws = torch.empty(max(256, lb.mivq_rabitq_search_workspace_bytes(a.nq, a.n, a.d, a.k)), dtype=torch.uint8,
                         device=dev)
        dd = torch.empty((a.nq, a.k), dtype=torch.float32, device=dev)
        ii = torch.empty((a.nq, a.k), dtype=torch.int32, device=dev)
        out[name] = (ws, dd, ii)

    def run(name):
        ws, dd, ii = out[name]
        rc = libs[name].mivq_rabitq_search(P(codes.data_ptr()), a.n, a.d, None, P(Q.data_ptr()), a.nq, a.qb,
                                           _native.METRIC_L2, a.k, 0, P(ws.data_ptr()), ws.numel(),
                                           P(dd.data_ptr()), P(ii.data_ptr()), P(st))
        assert rc == 0, rc

    for name in libs:
        run(name)
    torch.cuda.synchronize()
    same = "other" not in libs or bool(torch.equal(out["this"][1], out["other"][1]) and
                                       torch.equal(out["this"][2], out["other"][2]))
    print(f"identical ids and keys: {same}", flush=True)
    ts = {name: [] for name in libs}
    for _ in range(a.reps):
        for name in libs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(name)
            e1.record()
            torch.cuda.synchronize()
            ts[name].append(e0.elapsed_time(e1))
    for name in libs:
        t = sorted(ts[name])[len(ts[name]) // 2]
        print(f"rabitq_search {name}: median {t:.3f} ms = {a.nq / t * 1e3:.0f} queries/s "
              f"({a.nq} x {a.n} x {a.d}, qb {a.qb}, k {a.k})", flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
