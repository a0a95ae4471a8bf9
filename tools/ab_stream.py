"""Interleaved timing of the streaming encoders (SQ-8 f32, RaBitQ-1) across builds of libmivq.so.

usage: python tools/ab_stream.py A.so B.so ... [--n 1000000] [--d 3072] [--reps 10]
Prints per-call medians (HIP events) and whether each build's codes equal the first's.
"""
import argparse
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))
from haag_vq import _native  # noqa: E402
from tools.ab_lib import bind  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=3072)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = _native.require_device()
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    X = torch.randn((a.n, a.d), generator=g, device=dev, dtype=torch.float32)
    lo, hi = X.amin(0), X.amax(0)
    den = (hi - lo) + 1e-8
    libs = [bind(p) for p in a.libs]
    st = torch.cuda.current_stream().cuda_stream
    nb = (a.d + 7) // 8 + 8
    outs = {k: [torch.empty((a.n, a.d if k == "sq8" else nb), dtype=torch.uint8, device=dev) for _ in libs]
            for k in ("sq8", "rabitq1")}

    def call(k, i):
        if k == "sq8":
            rc = libs[i].mivq_sq_encode_f32(X.data_ptr(), a.n, a.d, lo.data_ptr(), den.data_ptr(), 8,
                                            outs[k][i].data_ptr(), st)
        else:
            rc = libs[i].mivq_rabitq_encode(X.data_ptr(), a.n, a.d, None, 1, outs[k][i].data_ptr(), st)
        assert rc == 0

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for k, bpv in (("sq8", 5 * a.d), ("rabitq1", 4 * a.d + nb)):
        times = [[] for _ in libs]
        for _ in range(3):
            for i in range(len(libs)):
                call(k, i)
        for _ in range(a.reps):
            for i in range(len(libs)):
                call(k, i)
                ev[0].record()
                call(k, i)
                ev[1].record()
                torch.cuda.synchronize()
                times[i].append(ev[0].elapsed_time(ev[1]))
        for i, p in enumerate(a.libs):
            t = sorted(times[i])[len(times[i]) // 2]
            print(f"{k:8s} {p:45s} median {t:.4f} ms  {a.n * bpv / t / 1e9:7.1f} GB/s = {a.n * bpv / t / 1e9 / 8000:.3f}"
                  f"  equal first: {torch.equal(outs[k][i], outs[k][0])}", flush=True)


if __name__ == "__main__":
    main()
