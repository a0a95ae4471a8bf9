"""Per-workgroup resolve list sizes of one mivq_pq_encode call (1M x 1536 Gaussian, PQ16): the
merged resolve's duration is that of its slowest workgroup, so max / mean of the per-workgroup
work says how much of it is imbalance (run on the GPU box)."""
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

n, d, M = 1_000_000, 1536, 16
dev = _native.require_device()
X = synth(n, d, 0, dev, kind="gaussian")
C = train_pq(X[:65536], M, 8, niter=25, seed=1234).contiguous()
prep = _native.pq_prepare(C, 8)
codes = _native.pq_encode(X, C, prep, 8)
torch.cuda.synchronize()
ws = _native.workspace(0, dev)
al = lambda v: (v + 255) // 256 * 256  # noqa: E731
off = al(n * M) + al(max(n * M * 8, (n + 31) // 32 * M * 4))
cnt = ws[off: off + 8 * 4096].view(torch.int32).cpu().numpy().reshape(-1, 2)
grid = int((cnt.sum(1) > 0).sum())
cnt = cnt[:256]
np_, nf = cnt[:, 0], cnt[:, 1]
work = np_ / 32 * 1.0 + nf / 32 * 4.0  # pair batch ~1, full batch ~4 (relative cost)
print("workgroups with items:", grid)
print(f"pairs per WG: mean {np_.mean():.0f} min {np_.min()} max {np_.max()}")
print(f"full  per WG: mean {nf.mean():.0f} min {nf.min()} max {nf.max()}")
print(f"weighted work max/mean {work.max() / work.mean():.3f}")
b = np.arange(256)
m_of = (b >> 3) % M  # wg_coords_of when the grid is a multiple of 8 M
for m in range(M):
    sel = m_of == m
    print(f"m={m:2d} pairs/WG {np_[sel].mean():7.0f}  full/WG {nf[sel].mean():7.0f}  work {work[sel].mean():6.1f}")
