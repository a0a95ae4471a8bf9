"""Where the bench's ADC wall time goes: the sharded call (LUT + search) timed by bench.timed at
several rep counts, beside its parts (mivq_adc_lut alone, mivq_adc_search alone) and the
per-call HIP-event means.

usage: python tools/probe_adc_wall.py [--n 1000000] [--d 1536] [--M 16] [--nq 1000] [--k 10]
Codes are the PQ encode of synthetic rows (bench.synth) with k-means codebooks, as in bench.py.
"""
import argparse
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))
from haag_vq import _native  # noqa: E402
from haag_vq.methods._kmeans import train_pq  # noqa: E402
from haag_vq.parallel import sharded  # noqa: E402
from bench import synth, timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=10)
    a = ap.parse_args()
    dev = _native.require_device()
    X = synth(a.n, a.d, 0, dev)
    C = train_pq(X[:65536], a.M, 8, niter=25, seed=1234).contiguous()
    codes = _native.pq_encode(X, C, _native.pq_prepare(C, 8), 8)
    del X
    Q = synth(a.nq, a.d, 7, dev)
    lut = _native.adc_lut(Q, C, 8)
    parts = {
        "sharded call (LUT + search)": lambda: sharded.sharded_adc_search(Q, C, codes, 8, a.k, 0),
        "mivq_adc_lut alone": lambda: _native.adc_lut(Q, C, 8),
        "mivq_adc_search alone": lambda: _native.adc_search(lut, codes, a.k, 8),
    }
    for name, fn in parts.items():
        for reps in (10, 30, 100):
            wall, ev = timed(fn, reps, 3)
            print(f"{name:30s} reps {reps:3d}: wall {wall * 1e3:.3f} ms/call ({a.nq / wall:,.0f} q/s), "
                  f"event mean {ev:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
