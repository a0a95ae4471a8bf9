"""CPU: the oracle is pinned against the reference's own fixtures and logged KATs."""

import json

import numpy as np
import pytest


def test_sq_oracle_matches_reference_fixtures(oracle, golden_dir):
    g = np.load(golden_dir / "sq_golden.npz")
    assert len(g["cases"]) == 18
    for tag in g["cases"]:
        tag = str(tag)
        X, lo, hi, codes, recon = (g[f"{tag}_{k}"] for k in ("X", "lo", "hi", "codes", "recon"))
        bits = int(tag.split("_b")[1])
        den = hi - lo + 1e-8
        c = oracle.sq_encode(X, lo, den, bits)
        np.testing.assert_array_equal(c, codes, err_msg=tag)
        r = oracle.sq_decode(c, X.shape[1], lo, den, bits)
        assert r.dtype == recon.dtype
        np.testing.assert_array_equal(r.view(np.uint8), recon.view(np.uint8), err_msg=tag)


def test_extrabitq_oracle_matches_reference_fixtures(oracle, golden_dir):
    e = np.load(golden_dir / "extrabitq_golden.npz")
    X = e["X"]
    for tag in e["cases"]:
        tag = str(tag)
        b = int(tag[1:])
        c, P, lv = oracle.extrabitq_fit(X, b)
        np.testing.assert_array_equal(c, e[f"{tag}_c"])
        np.testing.assert_array_equal(P, e[f"{tag}_P"])
        np.testing.assert_array_equal(lv, e[f"{tag}_levels"])
        codes = oracle.extrabitq_encode(X, c, P, lv, b)
        np.testing.assert_array_equal(codes, e[f"{tag}_codes"])
        np.testing.assert_array_equal(oracle.extrabitq_decode(codes, c, P, lv, b), e[f"{tag}_recon"])


@pytest.fixture(scope="module")
def dummy():
    """load_dummy_dataset(): np.random.seed(42); randn(10000, 1024) (datasets.py:79-81)."""
    np.random.seed(42)
    return np.random.randn(10000, 1024)


@pytest.fixture(scope="module")
def kat(golden_dir):
    return json.loads((golden_dir / "kat.json").read_text())


def _recall(gt, ret, k):
    return sum(len(set(gt[i, :k]) & set(ret[i, :k])) / k for i in range(len(gt))) / len(gt)


def test_sq8_kat_row38(oracle, dummy, kat):
    m = kat["38"]["metrics"]
    lo, hi, den = oracle.sq_fit(dummy)
    rec = oracle.sq_decode(oracle.sq_encode(dummy, lo, den, 8), 1024, lo, den, 8)
    dist = np.mean(np.sum((dummy - rec) ** 2, axis=1))
    # codes/reconstructions are bit-exact (fixtures); the logged fp64 mean differs by 1 ulp
    # (numpy's pairwise-summation blocking on the logging machine)
    assert abs(dist - m["reconstruction_distortion"]) <= 2 * np.spacing(m["reconstruction_distortion"])
    gt = oracle.exact_l2_topk(dummy[:100], dummy, 100)
    from sklearn.metrics import pairwise_distances

    ret = pairwise_distances(dummy[:100], rec).argsort(axis=1)
    assert _recall(gt, ret, 10) == pytest.approx(m["recall@10"], abs=1e-12)
    assert _recall(gt, ret, 100) == pytest.approx(m["recall@100"], abs=1e-12)


def test_rabitq_kat_row52(oracle, dummy, kat):
    m = kat["52"]["metrics"]
    codes = oracle.rabitq_encode(dummy.astype(np.float32))
    assert 4096 / codes.shape[1] == pytest.approx(m["compression_ratio"])
    rec = oracle.rabitq_decode(codes, 1024)
    dist = np.mean(np.sum((dummy - rec) ** 2, axis=1))
    assert dist == pytest.approx(m["reconstruction_distortion"], rel=1e-7)
    gt = oracle.exact_l2_topk(dummy[:100], dummy, 100)
    from sklearn.metrics import pairwise_distances

    ret = pairwise_distances(dummy[:100], rec).argsort(axis=1)
    assert _recall(gt, ret, 10) == pytest.approx(m["recall@10"], abs=1e-12)
    assert _recall(gt, ret, 100) == pytest.approx(m["recall@100"], abs=1e-12)


def test_pq_oracle_agrees_with_fp64_nearest_centroid(oracle):
    """Parity of the canonical PQ encode is unpinned vs faiss; any correct nearest-centroid
    implementation must agree with fp64 brute force wherever the top-2 gap is clear."""
    rng = np.random.default_rng(0)
    X = rng.standard_normal((600, 96)).astype(np.float32)
    C = rng.standard_normal((4, 256, 24)).astype(np.float32)
    codes = oracle.pq_encode(X, C)
    c64, gap = oracle.pq_encode_fp64(X, C)
    clear = gap > 1e-6
    assert clear.mean() > 0.95
    np.testing.assert_array_equal(codes[clear], c64[clear])


def test_pq_oracle_first_index_tie_break(oracle):
    C = np.zeros((1, 8, 4), np.float32)
    C[0, 2] = [1, 0, 0, 0]
    C[0, 5] = [1, 0, 0, 0]
    X = np.array([[1, 0, 0, 0], [0, 0, 0, 0], [np.nan, 0, 0, 0]], np.float32)
    codes = oracle.pq_encode(X, C)
    assert codes[:, 0].tolist() == [2, 0, 0]


def test_pq_pack_roundtrip(oracle):
    rng = np.random.default_rng(1)
    for M, nbits in ((8, 8), (4, 4), (10, 3), (7, 1), (5, 6)):
        u8 = rng.integers(0, 1 << nbits, size=(50, M)).astype(np.uint8)
        packed = oracle.pq_pack(u8, nbits)
        assert packed.shape[1] == (M * nbits + 7) // 8
        np.testing.assert_array_equal(oracle.pq_unpack(packed, M, nbits), u8)
    # faiss layout: sub-code m in bits [m*nbits, (m+1)*nbits), LSB first
    p = oracle.pq_pack(np.array([[1, 2]], np.uint8), 4)
    assert p.tolist() == [[0x21]]


def test_adc_oracle_equals_decode_then_exact(oracle):
    rng = np.random.default_rng(2)
    M, ksub, dsub = 4, 16, 8
    C = rng.standard_normal((M, ksub, dsub)).astype(np.float32)
    codes = rng.integers(0, ksub, size=(300, M)).astype(np.uint8)
    Q = rng.standard_normal((5, M * dsub)).astype(np.float32)
    d, i = oracle.adc_search(oracle.adc_lut(Q, C), codes, 10)
    Xh = oracle.pq_decode(codes, C).astype(np.float64)
    ref = ((Q[:, None, :].astype(np.float64) - Xh[None]) ** 2).sum(-1)
    np.testing.assert_allclose(d, np.take_along_axis(ref, i.astype(np.int64), 1), rtol=1e-5)
    assert np.all(np.diff(d, axis=1) >= 0)


def test_ivfpq_oracle_equals_decoded_distances(oracle):
    """The IVF-PQ restatement's expanded distance (coarse + tau + 2 S, include/mivq.h) equals
    ||q - (c_l + r_hat)||^2 (and -q.(c_l + r_hat) for IP) to fp32 rounding, with nprobe = K
    reaching every vector exactly once (faiss_ivfpq_index.py:46-76 semantics)."""
    rng = np.random.default_rng(4)
    n, d, K, M = 600, 32, 12, 8
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((7, d)).astype(np.float32)
    coarse = X[:K].copy()
    Cpq = (0.5 * rng.standard_normal((M, 256, d // M))).astype(np.float32)
    for metric in (1, 0):
        built = oracle.ivfpq_build(X, coarse, Cpq, metric)
        a, codes = built[0], built[1]
        xh = coarse[a.astype(np.int64)].astype(np.float64) + oracle.pq_decode(codes, Cpq).astype(np.float64)
        dd, ii = oracle.ivfpq_query(Q, coarse, Cpq, built, K, n, metric)
        assert sorted(ii[0].tolist()) == list(range(n))
        for q in range(len(Q)):
            if metric == 1:
                ref = ((Q[q].astype(np.float64) - xh[ii[q].astype(np.int64)]) ** 2).sum(1)
            else:
                ref = -(xh[ii[q].astype(np.int64)] @ Q[q].astype(np.float64))
            np.testing.assert_allclose(dd[q], ref, rtol=1e-4, atol=1e-3)


def test_bucket_sort_oracle_is_stable(oracle):
    a = np.array([3, 1, 3, 0, 1, 3], np.int32)
    off, order = oracle.bucket_sort(a, 5)
    assert off.tolist() == [0, 1, 3, 3, 6, 6]
    assert order.tolist() == [3, 1, 4, 0, 2, 5]


def test_rabitq_estimator_restatement_matches_fp64_formula():
    """oracle_rabitq_est (qb = 0) equals the RaBitQ estimator written out in fp64:
    ||r||^2 + ||q - c||^2 - 2 f1 <q - c, (2b - 1)/sqrt(d)>, and qb = 8 stays close to it."""
    import oracle as O

    rng = np.random.default_rng(5)
    n, nq, d = 200, 7, 64
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((nq, d)).astype(np.float32)
    c = X.mean(0).astype(np.float32)
    codes = O.rabitq_encode(X, c, metric=1)
    nb = d // 8
    bits = np.unpackbits(codes[:, :nb], axis=1, bitorder="little")[:, :d].astype(np.float64)
    f = codes[:, nb:].copy().view(np.float32).astype(np.float64)
    r = (Q - c).astype(np.float64)
    want = f[None, :, 0] + (r ** 2).sum(1)[:, None] - 2 * f[None, :, 1] * (r @ (2 * bits - 1).T) / np.sqrt(d)
    got0 = O.rabitq_est(codes, d, Q, c, qb=0, metric=1)
    np.testing.assert_allclose(got0, want, rtol=1e-4, atol=1e-3)
    got8 = O.rabitq_est(codes, d, Q, c, qb=8, metric=1)
    assert np.abs(got8 - want).max() < 0.05 * np.abs(want).max()
    # IP keys are the negated inner-product estimates 0.5 (pre - ||q||^2), f0 = ||r||^2 - ||x||^2
    codes_ip = O.rabitq_encode(X, c, metric=0)
    f_ip = codes_ip[:, nb:].copy().view(np.float32).astype(np.float64)
    pre = f_ip[None, :, 0] + (r ** 2).sum(1)[:, None] - 2 * f_ip[None, :, 1] * (r @ (2 * bits - 1).T) / np.sqrt(d)
    want_ip = 0.5 * (pre - (Q.astype(np.float64) ** 2).sum(1)[:, None])
    ip = O.rabitq_est(codes_ip, d, Q, c, qb=0, metric=0)
    np.testing.assert_allclose(ip, want_ip, rtol=1e-4, atol=1e-3)
    assert np.corrcoef(ip.ravel(), -(Q @ X.T).ravel())[0, 1] > 0.6  # 1-bit codes, d = 64


def test_oracle_asan_selftest():
    """the CPU oracle under -fsanitize=address,undefined (oracle/selftest.c runs
    every exported restatement at the shape edges; `make -C oracle asan` builds and runs it)."""
    import shutil
    from pathlib import Path
    import subprocess

    if shutil.which("gcc") is None and shutil.which("cc") is None:
        pytest.skip("no C compiler")
    p = subprocess.run(["make", "-s", "-C", str(Path(__file__).resolve().parents[1] / "oracle"), "asan"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "oracle selftest ok" in p.stdout
