"""Pairwise distance distortion — /root/reference/src/haag_vq/metrics/pairwise_distortion.py:37-140.

Same sampling (np.random.seed(seed); randint pairs; distinct), same statistic
|d(x_hat_i, x_hat_j) / (d(x_i, x_j) + 1e-10) - 1|.
"""

from typing import Dict

import numpy as np


def compute_pairwise_distortion(X_original, X_compressed_codes, model, num_pairs: int = 1000,
                                seed: int = 42) -> Dict[str, float]:
    np.random.seed(seed)
    N = len(X_original)
    idx1 = np.random.randint(0, N, num_pairs)
    idx2 = np.random.randint(0, N, num_pairs)
    mask = idx1 != idx2
    idx1, idx2 = idx1[mask], idx2[mask]
    if len(idx1) == 0:
        idx1 = np.arange(min(num_pairs, N // 2))
        idx2 = np.arange(min(num_pairs, N // 2)) + 1
    Xo = np.asarray(X_original)
    orig = np.linalg.norm(Xo[idx1] - Xo[idx2], axis=1)
    Xd = model.decompress(X_compressed_codes)
    if not isinstance(Xd, np.ndarray):
        Xd = Xd.detach().cpu().numpy()
    comp = np.linalg.norm(Xd[idx1] - Xd[idx2], axis=1)
    rel = np.abs(comp / (orig + 1e-10) - 1)
    return {"mean": float(np.mean(rel)), "median": float(np.median(rel)), "max": float(np.max(rel)),
            "std": float(np.std(rel)), "num_pairs": len(idx1)}


def compute_asymmetric_pairwise_distortion(X_original, X_compressed_codes, model, num_pairs: int = 1000,
                                           seed: int = 42) -> Dict[str, float]:
    return compute_pairwise_distortion(X_original, X_compressed_codes, model, num_pairs, seed)
