"""OPQ on the GPU: the hand-written rotation kernels against fp64 and against each other,
one step of the alternating optimisation against a numpy restatement, and OPQ codes against
the canonical encode of the rotated vectors (SURVEY.md §8a row a4, §8c "OPQ bit-exactness":
codes identical to the canonical encode of the GPU-rotated x, rotated values within 1e-5
relative)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

# |y - y64| <= TOL * ||x_row|| * ||a_col||: the fp32 rounding budget of a d-term dot product
TOL = 1e-5


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _orth(d, seed):
    q, _ = np.linalg.qr(np.random.default_rng(seed).standard_normal((d, d)))
    return q.astype(np.float32)


def _check(y, X, B):
    """y vs fp64 X @ B, relative to ||x_i|| ||b_j|| (NaN / inf rows must stay non-finite)."""
    ref = X.astype(np.float64) @ B.astype(np.float64)
    fin = np.isfinite(X).all(1)
    scale = np.linalg.norm(X[fin].astype(np.float64), axis=1)[:, None] * np.linalg.norm(B, axis=0)[None, :]
    err = np.abs(y[fin] - ref[fin])
    ok = err <= TOL * scale + 1e-30
    assert ok.all(), f"max rel err {np.max(err / np.maximum(scale, 1e-300)):.3e}"
    assert not np.isfinite(y[~fin]).all(axis=1).any()


@pytest.mark.parametrize("n,d", [(1000, 1536), (777, 1024), (400, 288), (300, 776), (65, 8), (1, 64)])
@pytest.mark.parametrize("transpose", [False, True])
def test_split_gemm_vs_fp64(dev, n, d, transpose):
    from haag_vq import _native

    rng = np.random.default_rng(n + d)
    X = rng.standard_normal((n, d)).astype(np.float32)
    if n > 10:
        X[3] *= 1e-20          # tiny row (per-row scale)
        X[4] *= 1e20           # huge row
        X[5] = 0.0
        X[6, 1] = np.nan
        X[7, 2] = np.inf
        X[8, ::3] *= 1e-6      # mixed magnitudes inside a row
    A = _orth(d, d) * (3.0 if d == 1024 else 1.0)  # also a non-orthonormal scale
    prep = _native.opq_prepare(_t(A, dev), transpose)
    assert prep is not None
    y = _native.opq_rotate_prepared(_t(X, dev), prep).cpu().numpy()
    _check(y, X, A if transpose else A.T)


@pytest.mark.parametrize("d", [1536, 288])
def test_split_gemm_row_scales_along_k(dev, d):
    """Per-row power-of-two scales against rows whose magnitude changes along k: growing 4x per
    32-dim K step, starting with zeros or with tiny values, nonzero only in the last dim,
    decreasing, one loud chunk mid-row -- next to ordinary rows of the same tile, both tile
    shapes (round 5 also measured scales found chunk by chunk inside the GEMM against these)."""
    from haag_vq import _native

    rng = np.random.default_rng(d)
    n = 300
    X = rng.standard_normal((n, d)).astype(np.float32)
    k = np.arange(d)
    X[10] *= (2.0 ** (2 * (k // 32) % 60)).astype(np.float32)   # grows 4x per chunk (wraps)
    X[11, :100] = 0.0
    X[11, 100:] *= 1e-30
    X[12, :32] *= 1e-30
    X[12, 32:] *= 1e30                                            # factor 2^-200: early terms vanish
    X[13, : d // 2] = 0.0
    X[14, :-1] = 0.0
    X[15] *= (2.0 ** -((k // 32) % 40)).astype(np.float32)        # decreasing
    X[16, 64:96] *= 1e6                                           # one loud chunk mid-row
    X[200] = X[10] * np.float32(1e-10)                            # the same pattern in another wave's rows
    A = _orth(d, d + 1)
    for transpose in (False, True):
        prep = _native.opq_prepare(_t(A, dev), transpose)
        y = _native.opq_rotate_prepared(_t(X, dev), prep).cpu().numpy()
        _check(y, X, A if transpose else A.T)


def test_split_gemm_chunk_boundary(dev):
    """More rows than one GEMM chunk (2^20 rows: the f16 planes of x are built per chunk):
    rows on both sides of the boundary and the ragged end match fp64."""
    from haag_vq import _native

    n, d = (1 << 20) + 300, 256
    g = torch.Generator(device=dev).manual_seed(7)
    X = torch.randn((n, d), device=dev, generator=g)
    A = _orth(d, 11)
    prep = _native.opq_prepare(_t(A, dev), False)
    y = _native.opq_rotate_prepared(X, prep)
    for lo, hi in ((0, 200), ((1 << 20) - 200, (1 << 20) + 200), (n - 100, n)):
        _check(y[lo:hi].cpu().numpy(), X[lo:hi].cpu().numpy(), A.T)


@pytest.mark.parametrize("n,d", [(500, 1536), (130, 100)])
def test_fp32_mfma_kernel_vs_fp64(dev, n, d):
    """mivq_opq_rotate: the plain fp32 MFMA kernel (any d, no preparation)."""
    from haag_vq import _native

    X = np.random.default_rng(1).standard_normal((n, d)).astype(np.float32)
    A = _orth(d, 2)
    for tr in (False, True):
        y = _native.opq_rotate(_t(X, dev), _t(A, dev), tr).cpu().numpy()
        _check(y, X, A if tr else A.T)


def test_prepare_rejects_d_not_multiple_of_8(dev):
    from haag_vq import _native

    assert _native.opq_prepare(_t(_orth(100, 0), dev)) is None


def test_opq_train_step_matches_restatement(dev, oracle):
    """One alternating-optimisation round (optimized_product_quantization.py:21-28 via faiss
    OPQMatrix::train): GPU vs numpy given the round's trained codebook."""
    from haag_vq.methods.optimized_product_quantization import OptimizedProductQuantizer

    rng = np.random.default_rng(4)
    X = (rng.standard_normal((3000, 64)) @ rng.standard_normal((64, 64))).astype(np.float32)
    opq = OptimizedProductQuantizer(M=8, B=8)
    Xd = _t(X, dev)
    A0 = opq.initial_rotation(64, dev)
    A1, C, Y, Yhat = opq.train_step(Xd, A0, None, 0)
    A0h, Yh, Ch = A0.cpu().numpy(), Y.cpu().numpy(), C.cpu().numpy()
    _check(Yh, X, A0h.T)                                                  # rotate
    codes = oracle.pq_encode(Yh, Ch)                                      # canonical encode
    np.testing.assert_array_equal(Yhat.cpu().numpy(), oracle.pq_decode(codes, Ch))  # bit-exact decode
    G = X.astype(np.float64).T @ oracle.pq_decode(codes, Ch).astype(np.float64)
    U, _, Vt = np.linalg.svd(G)
    np.testing.assert_allclose(A1.cpu().numpy(), (Vt.T @ U.T), atol=2e-6)  # Procrustes
    A1h = A1.cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(A1h @ A1h.T, np.eye(64), atol=1e-5)


def test_opq_codes_are_canonical_encode_of_rotated(dev, oracle):
    from haag_vq.methods.optimized_product_quantization import OptimizedProductQuantizer

    rng = np.random.default_rng(5)
    X = rng.standard_normal((4000, 256)).astype(np.float32)
    opq = OptimizedProductQuantizer(M=16, B=8)
    opq.niter = 3
    opq.fit(X)
    codes = opq.compress(X)
    Y = opq.opq.apply(X)                       # the GPU-rotated vectors
    C = np.stack(opq.inner.codebooks).astype(np.float32)
    np.testing.assert_array_equal(codes, oracle.pq_encode(Y, C))
    _check(Y, X, opq.opq.A.reshape(256, 256).T)
    rec = opq.decompress(codes)
    _check(rec, oracle.pq_decode(codes, C), opq.opq.A.reshape(256, 256))


@pytest.mark.parametrize("n,d", [(5000, 200), (70_000, 256), (33, 1536), (0, 64)])
def test_opq_gram_matches_fp64(dev, n, d):
    """mivq_opq_gram: G = X^T Y in fp64 (split over rows, parts added in order) vs numpy fp64;
    every product is exact, only the summation order differs."""
    from haag_vq import _native

    rng = np.random.default_rng(n + d)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Y = (rng.standard_normal((n, d)) * rng.uniform(0.01, 100, d)).astype(np.float32)
    G = _native.opq_gram(_t(X, dev), _t(Y, dev)).cpu().numpy()
    ref = X.astype(np.float64).T @ Y.astype(np.float64)
    bound = 1e-13 * (np.abs(X).astype(np.float64).T @ np.abs(Y).astype(np.float64)) + 1e-300
    assert np.all(np.abs(G - ref) <= bound * max(1, n) ** 0.5 + 0)


def test_polar_factor_newton_schulz(dev):
    """polar_factor: the orthogonal polar factor U V^T of an ill-conditioned G (kappa ~ 1e4)
    from the Newton-Schulz iteration on the fp64 MFMA GEMM, vs numpy's SVD; a rank-deficient
    G takes the SVD fallback and still returns an orthogonal matrix."""
    from haag_vq.methods.optimized_product_quantization import polar_factor

    rng = np.random.default_rng(8)
    d = 300
    U, _ = np.linalg.qr(rng.standard_normal((d, d)))
    V, _ = np.linalg.qr(rng.standard_normal((d, d)))
    S = np.logspace(0, -4, d)
    G = (U * S) @ V.T
    info = {}
    Q = polar_factor(_t(G, dev), info=info).cpu().numpy()
    assert info["path"] == "newton-schulz", info
    np.testing.assert_allclose(Q, U @ V.T, atol=1e-9)
    np.testing.assert_allclose(Q.T @ Q, np.eye(d), atol=1e-12)
    S[-3:] = 0.0  # rank deficient: Newton-Schulz keeps the zero singular values -> fallback
    Gd = (U * S) @ V.T
    info = {}
    Qd = polar_factor(_t(Gd, dev), info=info).cpu().numpy()
    assert info["path"] == "svd" and info["iters"] < 45, info  # the stall is seen early
    np.testing.assert_allclose(Qd.T @ Qd, np.eye(d), atol=1e-10)
    np.testing.assert_allclose(Qd @ (Qd.T @ Gd), Gd, atol=1e-10)


@pytest.mark.gpu
def test_polar_factor_small_singular_tail_stays_on_newton_schulz(dev):
    """ones plus 8 singular values at 1e-3 (a tail of low-variance directions) hold
    ||Q^T Q - I|| near sqrt(8) for ~17 steps while they grow 1.5x per step.  That is not rank
    deficiency: the iteration must go on to the polar factor, not to the SVD."""
    from haag_vq.methods.optimized_product_quantization import polar_factor

    rng = np.random.default_rng(12)
    d = 128
    U, _ = np.linalg.qr(rng.standard_normal((d, d)))
    V, _ = np.linalg.qr(rng.standard_normal((d, d)))
    S = np.ones(d)
    S[-8:] = 1e-3
    G = (U * S) @ V.T
    info = {}
    Q = polar_factor(_t(G, dev), info=info).cpu().numpy()
    assert info["path"] == "newton-schulz", info
    np.testing.assert_allclose(Q, U @ V.T, atol=1e-9)


def test_polar_factor_top_vector_orthogonal_to_ones(dev):
    """G whose dominant right singular vector is orthogonal to the all-ones vector
    and whose top two singular values are 2 : 1.  A start scale estimated from below (a power
    iteration from ones / sqrt(d)) would put the top value near 1.8 > sqrt(3), where
    Newton-Schulz converges to -1: an orthogonal matrix that is NOT the polar factor.  The
    upper-bound scale must give U V^T."""
    from haag_vq.methods.optimized_product_quantization import polar_factor

    rng = np.random.default_rng(11)
    d = 64
    U, _ = np.linalg.qr(rng.standard_normal((d, d)))
    v1 = np.zeros(d)
    v1[0], v1[1] = 2 ** -0.5, -(2 ** -0.5)  # orthogonal to ones
    V = np.linalg.qr(np.column_stack([v1, rng.standard_normal((d, d - 1))]))[0]  # V[:, 0] = +-v1
    assert abs(V[:, 0] @ np.ones(d)) < 1e-12
    S = np.ones(d)
    S[0] = 2.0
    G = (U * S) @ V.T
    Q = polar_factor(_t(G, dev)).cpu().numpy()
    np.testing.assert_allclose(Q, U @ V.T, atol=1e-9)
    # Q^T G is the symmetric positive definite factor V S V^T
    P = Q.T @ G
    np.testing.assert_allclose(P, P.T, atol=1e-9)
    assert np.linalg.eigvalsh((P + P.T) / 2).min() > 0.5
