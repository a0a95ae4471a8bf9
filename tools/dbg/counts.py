"""Per-workgroup resolve list sizes of one mivq_pq_encode call (cs path): the merged resolve's
duration is that of its slowest workgroup, so max / mean of the per-workgroup work says how much
of it is imbalance, and the totals say how many row-subspaces the filter left (run on the GPU box).

usage: python tools/dbg/counts.py [n] [d] [M]   (defaults 1000000 1536 16; Gaussian rows)
"""
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 1536
M = int(sys.argv[3]) if len(sys.argv) > 3 else 16
dev = _native.require_device()
X = synth(n, d, 0, dev, kind="gaussian")
C = train_pq(X[:65536], M, 8, niter=25, seed=1234).contiguous()
prep = _native.pq_prepare(C, 8)
lib = _native.load_library()
nb = lib.mivq_pq_encode_workspace_bytes(n, d, M, 8)
ws = torch.zeros(nb, dtype=torch.uint8, device=dev)  # counts of unused workgroups stay 0
codes = torch.empty((n, M), dtype=torch.uint8, device=dev)
_native._call("mivq_pq_encode", _native._ptr(X), n, d, M, 8, _native._ptr(C), _native._ptr(prep), _native._ptr(ws),
              ws.numel(), _native._ptr(codes), 0, _native._stream())
torch.cuda.synchronize()
al = lambda v: (v + 255) // 256 * 256  # noqa: E731 (mivq_pq_encode's workspace layout)
off = al(n * M) + al(max(n * M * 8, (n + 31) // 32 * M * 4))
cnt = ws[off: off + al((n + 127) // 128 * M * 8)].view(torch.int32).cpu().numpy().reshape(-1, 2)
used = cnt.sum(1) > 0
np_, nf = cnt[used, 0], cnt[used, 1]
print(f"n={n} d={d} M={M} dsub={d // M}: workgroups with items {int(used.sum())}")
print(f"pair items {np_.sum()} ({np_.sum() / (n * M):.4%} of row-subspaces), "
      f"full items {nf.sum()} ({nf.sum() / (n * M):.4%})")
print(f"pairs per WG: mean {np_.mean():.0f} max {np_.max()}   full per WG: mean {nf.mean():.0f} max {nf.max()}")
work = np_ / 32 * 1.0 + nf / 32 * 4.0  # pair batch ~1, full batch ~4 (relative cost)
print(f"weighted work max/mean {work.max() / work.mean():.3f}")
