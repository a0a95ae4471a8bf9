"""Interleaved timing of mivq_opq_rotate_prepared across builds of libmivq.so (same data).

usage: python tools/ab_opq.py A.so B.so ... [--n 1000000] [--d 1536] [--reps 8]
Prints per-call medians (HIP events), TF/s (2 n d^2 fp32-accurate flops) and whether each
build's output equals the first build's bit for bit.
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
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    dev = _native.require_device()
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    X = torch.randn((a.n, a.d), generator=g, device=dev, dtype=torch.float32)
    A, _ = torch.linalg.qr(torch.randn((a.d, a.d), generator=g, device=dev, dtype=torch.float64))
    A = A.float().contiguous()
    libs = [bind(p) for p in a.libs]
    st = torch.cuda.current_stream().cuda_stream
    preps, ws, outs = [], [], []
    for lib in libs:
        prep = torch.empty(lib.mivq_opq_prep_bytes(a.d), dtype=torch.uint8, device=dev)
        assert lib.mivq_opq_prepare(A.data_ptr(), a.d, 0, prep.data_ptr(), st) == 0
        preps.append(prep)
        ws.append(torch.empty(lib.mivq_opq_rotate_workspace_bytes(a.n, a.d), dtype=torch.uint8, device=dev))
        outs.append(torch.empty_like(X))

    def call(i):
        rc = libs[i].mivq_opq_rotate_prepared(X.data_ptr(), a.n, a.d, preps[i].data_ptr(), ws[i].data_ptr(),
                                              ws[i].numel(), outs[i].data_ptr(), st)
        assert rc == 0, libs[i].mivq_last_error()

    for _ in range(2):
        for i in range(len(libs)):
            call(i)
    times = [[] for _ in libs]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(a.reps):
        for i in range(len(libs)):
            call(i)
            ev[0].record()
            call(i)
            ev[1].record()
            torch.cuda.synchronize()
            times[i].append(ev[0].elapsed_time(ev[1]))
    ns = min(a.n, 20000)
    ref = X[:ns].double() @ A.double().T
    for i, p in enumerate(a.libs):
        t = sorted(times[i])[len(times[i]) // 2]
        err = float(((outs[i][:ns].double() - ref).abs().max() / ref.abs().max()).item())
        print(f"{p:45s} median {t:8.3f} ms  {2 * a.n * a.d * a.d / t / 1e9:7.1f} TF/s  equal first: "
              f"{torch.equal(outs[i], outs[0])}  max rel err vs fp64 {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
