"""Start / end times of every filter workgroup of one mivq_pq_encode call (1M x 1536 Gaussian,
PQ16), from a library built with -DMIVQ_CS_TIMESTAMPS (wall_clock64, 100 MHz): how ragged the
filter's ending is, i.e. how much of the resolve a persistent tail could hide (GPU box).
Build: hipcc <Makefile flags> -DMIVQ_CS_TIMESTAMPS -c pq_encode_cs.hip, link with the other
objects into tools/build/lib_ts.so, run with MIVQ_LIB=$PWD/tools/build/lib_ts.so."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))
from haag_vq import _native  # noqa: E402
from haag_vq.methods._kmeans import train_pq  # noqa: E402
from bench import synth  # noqa: E402

assert "lib_ts" in os.environ.get("MIVQ_LIB", ""), "run with MIVQ_LIB=tools/build/lib_ts.so"
n, d, M = 1_000_000, 1536, 16
dev = _native.require_device()
X = synth(n, d, 0, dev, kind="gaussian")
C = train_pq(X[:65536], M, 8, niter=25, seed=1234).contiguous()
prep = _native.pq_prepare(C, 8)
out = torch.empty((n, M), dtype=torch.uint8, device=dev)
al = lambda v: (v + 255) // 256 * 256  # noqa: E731
off = al(n * M) + al(max(n * M * 8, (n + 31) // 32 * M * 4)) + al((n + 127) // 128 * M * 8)
for call in range(60):
    _native.pq_encode(X, C, prep, 8, out=out)
    if call in (5, 30, 59):
        torch.cuda.synchronize()
        ws = _native.workspace(0, dev)
        t = ws[off: off + 16 * 256].view(torch.int64).cpu().numpy().reshape(-1, 2).astype(np.float64) / 100.0  # us
        t -= t[:, 0].min()
        s, e = t[:, 0], t[:, 1]
        q = np.percentile(e, [0, 10, 50, 90, 100])
        print(f"call {call}: starts {s.min():.1f}..{s.max():.1f} us; ends min/p10/p50/p90/max "
              f"{' / '.join(f'{v:.0f}' for v in q)} us; mean idle before the last end {np.mean(e.max() - e):.0f} us",
              flush=True)
        xcd = np.arange(256) % 8
        print("  end by XCD (mean us):", " ".join(f"{e[xcd == x].mean():.0f}" for x in range(8)), flush=True)
        chunk = (np.arange(256) >> 3) // M * 8 + (np.arange(256) & 7)
        print("  end by chunk (mean us):", " ".join(f"{e[chunk == c].mean():.0f}" for c in range(16)), flush=True)
