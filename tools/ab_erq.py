"""Interleaved A/B of mivq_extrabitq_rotate (erq_rotate_kernel) between two builds of libmivq.so.

usage: python tools/ab_erq.py OTHER.so [--n 200000] [--d 3072] [--reps 6]
"this" = the in-tree library.  Same inputs for both, outputs compared bit for bit; prints per-call
medians (HIP events, alternating calls) and the fp64-MFMA rate (2 n d^2 FLOP per call).
"""
import argparse
import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT / "tools"))
from ab_lib import bind  # noqa: E402
from haag_vq import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("other")
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--d", type=int, default=3072)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    libs = {"this": bind(_native.LIB_PATH), "other": bind(Path(a.other).resolve())}
    g = torch.Generator(device=dev).manual_seed(5)
    o = torch.randn((a.n, a.d), dtype=torch.float64, device=dev, generator=g)
    P = torch.linalg.qr(torch.randn((a.d, a.d), dtype=torch.float64, device=dev, generator=g))[0].contiguous()
    outs = {k: torch.empty((a.n, a.d), dtype=torch.float64, device=dev) for k in libs}
    st = torch.cuda.current_stream().cuda_stream
    P_ = ctypes.c_void_p

    def run(k, transpose=0):
        rc = libs[k].mivq_extrabitq_rotate(P_(o.data_ptr()), a.n, a.d, P_(P.data_ptr()), transpose,
                                           P_(outs[k].data_ptr()), P_(st))
        assert rc == 0, rc

    for k in libs:
        run(k)
    torch.cuda.synchronize()
    same = bool(torch.equal(outs["this"], outs["other"]))
    res = {k: [] for k in libs}
    for _ in range(a.reps):
        for k in libs:
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_.record()
            run(k)
            e_.record()
            torch.cuda.synchronize()
            res[k].append(s_.elapsed_time(e_))
    flop = 2.0 * a.n * a.d * a.d
    for k in libs:
        t = sorted(res[k])
        med = t[len(t) // 2]
        print(f"AB erq {k}: median {med:.2f} ms  min {t[0]:.2f}  = {flop / (med * 1e-3) / 1e12:.1f} TF/s", flush=True)
    print(f"outputs identical: {same}", flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
