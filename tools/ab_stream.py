"""Interleaved A/B of the streaming encoders (mivq_sq_encode_f32 8-bit, mivq_rabitq_encode) between
two builds of libmivq.so: same inputs, outputs compared byte for byte.

usage: python tools/ab_stream.py OTHER.so [--kind sq8|rabitq1] [--n 1000000] [--d 3072] [--reps 10]
"this" = the in-tree library.  Prints per-call medians (HIP events, alternating calls) and the
HBM rate of the algorithmic bytes (4 d read + the code row written per vector).
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
    ap.add_argument("--kind", choices=("sq8", "rabitq1"), default="rabitq1")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=3072)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    libs = {"this": bind(_native.LIB_PATH), "other": bind(Path(a.other).resolve())}
    g = torch.Generator(device=dev).manual_seed(2)
    X = torch.randn((a.n, a.d), generator=g, device=dev, dtype=torch.float32)
    st = torch.cuda.current_stream().cuda_stream
    P = ctypes.c_void_p
    if a.kind == "sq8":
        lo = X.amin(0).contiguous()
        den = ((X.amax(0) - lo) + 1e-8).contiguous()
        cs, bpv = a.d, 5 * a.d
    else:
        cs, bpv = (a.d + 7) // 8 + 8, 4 * a.d + (a.d + 7) // 8 + 8
    outs = {k: torch.empty((a.n, cs), dtype=torch.uint8, device=dev) for k in libs}

    def run(k):
        if a.kind == "sq8":
            rc = libs[k].mivq_sq_encode_f32(P(X.data_ptr()), a.n, a.d, P(lo.data_ptr()), P(den.data_ptr()), 8,
                                           P(outs[k].data_ptr()), P(st))
        else:
            rc = libs[k].mivq_rabitq_encode(P(X.data_ptr()), a.n, a.d, None, _native.METRIC_L2,
                                           P(outs[k].data_ptr()), P(st))
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
    for k in libs:
        t = sorted(res[k])
        med = t[len(t) // 2]
        print(f"AB {a.kind} {k}: median {med:.3f} ms  min {t[0]:.3f}  = {a.n * bpv / (med * 1e-3) / 8e12:.3f} of 8 TB/s",
              flush=True)
    print(f"outputs identical: {same}", flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
