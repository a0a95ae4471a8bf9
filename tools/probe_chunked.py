"""One mivq_pq_encode call over N rows vs the same rows encoded as consecutive row slices of S
rows each (same stream, back to back), interleaved; checks the codes are identical.

usage: python tools/probe_chunked.py [N] [S ...]   (defaults 10000000 and 1048576 2097152 524288)
"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from haag_vq import _native  # noqa: E402
from haag_vq.methods._kmeans import train_pq  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    slices = [int(v) for v in sys.argv[2:]] or [1 << 20, 1 << 21, 1 << 19]
    dev = _native.require_device()
    X = bench.synth(n, 1536, 11, dev)
    C = train_pq(X[:65536], 16, 8, niter=25, seed=1234, exact_assign=True).contiguous()
    prep = _native.pq_prepare(C, 8)
    ref = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    out = torch.empty_like(ref)

    def whole():
        _native.pq_encode(X, C, prep, 8, out=ref)

    def chunked(s):
        for r0 in range(0, n, s):
            r1 = min(n, r0 + s)
            _native.pq_encode(X[r0:r1], C, prep, 8, out=out[r0:r1])

    fns = {"whole": whole, **{f"slices of {s}": (lambda s=s: chunked(s)) for s in slices}}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    # settle the power state, then interleave
    for _ in range(3):
        whole()
    times = {k: [] for k in fns}
    for _ in range(5):
        for k, f in fns.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); f(); b.record()
            torch.cuda.synchronize()
            times[k].append(a.elapsed_time(b))
    for k, t in times.items():
        t = sorted(t)
        print(f"{k:22s} median {t[len(t) // 2]:8.3f} ms  min {t[0]:8.3f}  -> {n / t[len(t) // 2] / 1e3:7.1f} M vec/s "
              f"= {n * 6160 / (t[len(t) // 2] * 1e-3) / 8e12:.3f} of 8 TB/s", flush=True)
    print("codes equal:", bool(torch.equal(ref, out)), flush=True)


if __name__ == "__main__":
    main()
