"""Times the PQ encode paths on one Gaussian block: AUTO (MFMA filter when it applies), the
tiled exact kernel (FORCE_EXACT) and the lane-per-row exact kernel (FORCE_EXACT|LEGACY_EXACT),
for several M at D = 1536; checks that all three give the same codes.

usage: python tools/probe_exact.py [n] [M ...]
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
    fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    Ms = [int(v) for v in sys.argv[2:]] or [4, 8, 16]
    dev = _native.require_device()
    X = bench.synth(n, 1536, 0, dev)
    for M in Ms:
        C = train_pq(X[:32768], M, 8, niter=4, seed=1234, exact_assign=True).contiguous()
        prep = _native.pq_prepare(C, 8)
        outs = {}
        for name, kw in (("auto", {}), ("exact_tiled", {"exact": True}),
                         ("exact_lane", {"exact": True, "flags_extra": _native.MIVQ_PQ_LEGACY_EXACT})):
            out = torch.empty((n, M), dtype=torch.uint8, device=dev)
            reps = 3 if name == "exact_lane" else 10
            ms = timed(lambda: _native.pq_encode(X, C, prep, 8, out=out, **kw), reps)
            outs[name] = out
            print(f"M={M:3d} dsub={1536 // M:4d} {name:12s} {ms:9.3f} ms  {n / ms / 1e3:8.1f} M vec/s", flush=True)
        print(f"M={M:3d} codes equal: tiled==auto {torch.equal(outs['exact_tiled'], outs['auto'])} "
              f"lane==auto {torch.equal(outs['exact_lane'], outs['auto'])}", flush=True)


if __name__ == "__main__":
    main()
