"""Run the prepared OPQ rotation (1M x 1536 by default) a few times: a short program for
rocprofv3 --pmc / --kernel-trace passes over the split-f16 rotation kernels.

usage: python tools/opq_probe.py [--n 1000000] [--d 1536] [--reps 5]
"""
import argparse
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
from haag_vq import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lib-gemm", action="store_true",
                    help="also time plain f16 / bf16 / fp32 library GEMMs (torch.matmul) of the same shape")
    a = ap.parse_args()
    dev = _native.require_device()
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn((a.n, a.d), device=dev, generator=g)
    A, _ = torch.linalg.qr(torch.randn((a.d, a.d), device=dev, generator=g, dtype=torch.float64))
    A = A.float().contiguous()
    prep = _native.opq_prepare(A, transpose=False)
    y = torch.empty_like(x)
    for _ in range(2):
        _native.opq_rotate_prepared(x, prep, y)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        _native.opq_rotate_prepared(x, prep, y)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.reps
    print(f"opq rotate {a.n}x{a.d}: {ms:.3f} ms/call = {2 * a.n * a.d * a.d / (ms * 1e-3) / 1e12:.1f} TF/s", flush=True)
    if a.lib_gemm:  # yardsticks: one library GEMM of this shape in f16 / bf16 / fp32
        for dt in (torch.float16, torch.bfloat16, torch.float32):
            xh, bh = x.to(dt), A.to(dt)
            for _ in range(2):
                torch.matmul(xh, bh)
            torch.cuda.synchronize()
            s.record()
            for _ in range(a.reps):
                torch.matmul(xh, bh)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.reps
            print(f"library {dt} GEMM {a.n}x{a.d}x{a.d}: {ms:.3f} ms = "
                  f"{2 * a.n * a.d * a.d / (ms * 1e-3) / 1e12:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
