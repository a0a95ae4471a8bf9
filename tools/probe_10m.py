"""Why does one 10M-row PQ16 encode cost more per row than a 1M-row one?  Times, on the same
10M x 1536 Gaussian block: one 10M call; ten 1M calls over its slices; 1M calls alone; 2M and
5M calls.  Prints ms per 1M rows for each (after warm-up, sustained back to back).

usage: python tools/probe_10m.py [n_total]
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import bench  # noqa: E402
from haag_vq import _native  # noqa: E402
from haag_vq.methods._kmeans import train_pq  # noqa: E402


def timed(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    dev = _native.require_device()
    X = bench.synth(n, 1536, 0, dev)
    C = train_pq(X[:65536], 16, 8, niter=10, seed=1234, exact_assign=True).contiguous()
    prep = _native.pq_prepare(C, 8)
    out = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    M1 = 1_000_000

    def call(a, b):
        _native.pq_encode(X[a:b], C, prep, 8, out=out[a:b])

    for _ in range(3):
        call(0, n)
    timed(lambda: call(0, M1), 40)  # settle
    res = {}
    res["10M_one_call"] = timed(lambda: call(0, n), 5) / (n / M1)
    res["10x1M_slices"] = timed(lambda: [call(i, i + M1) for i in range(0, n, M1)], 5) / (n / M1)
    res["1M_alone_x50"] = timed(lambda: call(0, M1), 50)
    res["2M_one_call"] = timed(lambda: call(0, 2 * M1), 20) / 2
    res["5M_one_call"] = timed(lambda: call(0, 5 * M1), 8) / 5
    res["10M_one_call_again"] = timed(lambda: call(0, n), 5) / (n / M1)
    for k, v in res.items():
        print(f"{k:22s} {v:8.4f} ms per 1M rows   {1e3 / v:8.1f} M vec/s", flush=True)


if __name__ == "__main__":
    main()
