"""Interleaved timing of mivq_pq_encode across several builds of libmivq.so (same data).

usage: python tools/ab_multi.py A.so B.so ... [--n 1000000] [--reps 10] [--data gaussian]
Prints the per-call median (HIP events) of each build and whether its codes equal the first's.
"""
import argparse
import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))
from haag_vq import _native  # noqa: E402
from haag_vq.methods._kmeans import train_pq  # noqa: E402
from bench import synth  # noqa: E402
from tools.ab_lib import bind  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--data", default="gaussian")
    a = ap.parse_args()
    dev = _native.require_device()
    X = synth(a.n, a.d, 0, dev, kind=a.data)
    C = train_pq(X[:65536], a.M, 8, niter=10, seed=1234, exact_assign=True).contiguous()
    libs = [bind(p) for p in a.libs]
    st = torch.cuda.current_stream().cuda_stream
    outs, preps, ws = [], [], []
    for lib in libs:
        prep = torch.empty(lib.mivq_pq_prep_bytes(a.d, a.M, 8), dtype=torch.uint8, device=dev)
        assert lib.mivq_pq_prepare(C.data_ptr(), a.d, a.M, 8, prep.data_ptr(), st) == 0
        nb = lib.mivq_pq_encode_workspace_bytes(a.n, a.d, a.M, 8)
        preps.append(prep)
        ws.append(torch.empty(nb, dtype=torch.uint8, device=dev))
        outs.append(torch.empty((a.n, a.M), dtype=torch.uint8, device=dev))

    def call(i):
        rc = libs[i].mivq_pq_encode(X.data_ptr(), a.n, a.d, a.M, 8, C.data_ptr(), preps[i].data_ptr(), ws[i].data_ptr(),
                                    ws[i].numel(), outs[i].data_ptr(), 0, st)
        assert rc == 0, libs[i].mivq_last_error()

    for _ in range(3):
        for i in range(len(libs)):
            call(i)
    times = [[] for _ in libs]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(a.reps):
        for i in range(len(libs)):
            for _ in range(3):
                call(i)
            ev[0].record()
            call(i)
            ev[1].record()
            torch.cuda.synchronize()
            times[i].append(ev[0].elapsed_time(ev[1]))
    for i, p in enumerate(a.libs):
        t = sorted(times[i])[len(times[i]) // 2]
        same = torch.equal(outs[i], outs[0])
        print(f"{p:50s} median {t:.4f} ms   {a.n / t / 1e3:8.1f} M vec/s   codes equal first: {same}", flush=True)


if __name__ == "__main__":
    main()
