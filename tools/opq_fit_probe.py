"""The OPQ32 fit of bench.py's opq32 leg (1M x 1536 synthetic rows, the first 65,536 as the
training sample, 4 outer iterations), timed: a short program for rocprofv3 --kernel-trace
--stats, whose kernel list shows which kernels the training runs (round 4: no rocsolver SVD and
no rocBLAS DGEMM -- mivq_opq_gram + the Newton-Schulz polar factor on the fp64 MFMA GEMM).

usage: python tools/opq_fit_probe.py [--n 65536] [--d 1536] [--M 32] [--iters 4]
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))
from haag_vq import _native  # noqa: E402
from haag_vq.methods.optimized_product_quantization import OptimizedProductQuantizer  # noqa: E402
from bench import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--M", type=int, default=32)
    ap.add_argument("--iters", type=int, default=4)
    a = ap.parse_args()
    dev = _native.require_device()
    X = synth(a.n, a.d, seed=0, dev=dev, kind="gaussian")
    for rep in range(2):
        opq = OptimizedProductQuantizer(M=a.M, B=8)
        opq.niter = a.iters
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        opq.fit(X)
        torch.cuda.synchronize()
        A = opq.opq.A_device.cpu().double().numpy()  # the check on the host: no device BLAS in the trace
        orth = float(abs(A @ A.T - np.eye(a.d)).max()) if rep else 0.0
        print(f"OPQ{a.M} fit {a.n}x{a.d}, {a.iters} outer iterations: {time.perf_counter() - t0:.3f} s"
              + (f"; max |A A^T - I| {orth:.2e}" if rep else ""), flush=True)


if __name__ == "__main__":
    main()
