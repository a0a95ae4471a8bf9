"""Per-subspace k-means (PQ codebook training) on the MI355X.

Replaces faiss' ``ProductQuantizer.train`` as called by ProductQuantizer.fit
(/root/reference/src/haag_vq/methods/product_quantization.py:67-68) with the same
algorithm shape faiss documents for its default ``Clustering``: a random training sample
of at most ``max_points_per_centroid * ksub`` rows (seed 1234), initial centroids drawn
from the sample, ``niter`` Lloyd iterations, and empty clusters re-seeded by splitting a
populated one with a symmetric 1/1024 perturbation.  All M subspaces train together:
the assignment step IS ``mivq_pq_encode`` (the canonical nearest-centroid kernel) and the
update is ``mivq_kmeans_update`` (deterministic ascending-row sums), so a fit is
bit-reproducible for a given input and seed.  faiss' own k-means is unpinned here (the
package is absent), so the codebooks are not claimed to equal faiss'.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _native

EPS = 1.0 / 1024.0


def _split_empty(C: np.ndarray, counts: np.ndarray, rng: np.random.Generator, n: int) -> int:
    """faiss-style split of empty clusters, per subspace, in place.  Returns #splits."""
    M, ksub, _ = C.shape
    nsplit = 0
    for m in range(M):
        cnt = counts[m].astype(np.float64)
        for ci in range(ksub):
            if cnt[ci] != 0:
                continue
            cj = 0
            denom = max(1.0, float(n - ksub))
            for _ in range(64 * ksub):  # bounded: faiss loops until a draw succeeds
                p = (cnt[cj] - 1.0) / denom
                if rng.random() < p:
                    break
                cj = (cj + 1) % ksub
            else:
                cj = int(np.argmax(cnt))
            C[m, ci] = C[m, cj]
            sign = np.where(np.arange(C.shape[2]) % 2 == 0, 1.0, -1.0).astype(np.float32)
            C[m, ci] *= (1.0 + EPS * sign).astype(np.float32)
            C[m, cj] *= (1.0 - EPS * sign).astype(np.float32)
            cnt[ci] = np.floor(cnt[cj] / 2)
            cnt[cj] -= cnt[ci]
            nsplit += 1
    return nsplit


def train_pq(X: torch.Tensor, M: int, nbits: int, niter: int = 25, seed: int = 1234,
             max_points_per_centroid: int = 256, init: torch.Tensor | None = None,
             exact_assign: bool = False) -> torch.Tensor:
    """Train (M, 2**nbits, d/M) f32 centroids on device rows X (n, d).

    exact_assign: assign with the exact VALU encode instead of the MFMA filter path (same
    codes, so the same centroids; bench.py uses it to keep its profile free of training
    launches of the filter kernels).
    """
    n, d = X.shape
    if d % M != 0:
        raise AssertionError("D must be divisible by M (number of subquantizers)")
    ksub = 1 << nbits
    dsub = d // M
    if n < ksub:
        raise RuntimeError(
            f"Number of training points ({n}) should be at least as large as number of clusters ({ksub})"
        )
    rng = np.random.default_rng(seed)
    max_n = max_points_per_centroid * ksub
    if n > max_n:
        sel = rng.permutation(n)[:max_n]
        Xt = X[torch.from_numpy(np.sort(sel)).to(X.device)].contiguous()
    else:
        Xt = X.contiguous()
    nt = Xt.shape[0]
    if init is None:
        pick = np.sort(rng.permutation(nt)[:ksub])
        C = Xt[torch.from_numpy(pick).to(X.device)].reshape(ksub, M, dsub).permute(1, 0, 2).contiguous()
    else:
        C = init.to(device=X.device, dtype=torch.float32).contiguous().clone()
    counts = torch.empty((M, ksub), dtype=torch.int32, device=X.device)
    for _ in range(niter):
        prep = _native.pq_prepare(C, nbits)
        codes = _native.pq_encode(Xt, C, prep, nbits, exact=exact_assign)
        assign = codes if nbits == 8 else _native.pq_unpack(codes, M, nbits)
        _native.kmeans_update(Xt, assign, C, counts)
        cnt = counts.cpu().numpy()
        if (cnt == 0).any():
            Ch = C.cpu().numpy()
            _split_empty(Ch, cnt, rng, nt)
            C = torch.from_numpy(Ch).to(X.device).contiguous()
    return C
