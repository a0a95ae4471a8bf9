"""Reconstruction distortion — /root/reference/src/haag_vq/metrics/distortion.py:4-7."""

import numpy as np


def compute_distortion(X_original, X_compressed_codes, model):
    """mean over vectors of sum over dims of (x - x_hat)^2 (the sweep's per-vector SSE)."""
    X_rec = model.decompress(X_compressed_codes)
    if not isinstance(X_rec, np.ndarray):
        X_rec = X_rec.detach().cpu().numpy()
    diffs = np.asarray(X_original) - X_rec
    return np.mean(np.sum(diffs ** 2, axis=1))
