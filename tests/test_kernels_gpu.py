"""GPU parity: every libmivq entry point against the CPU oracle (bit-exact where the
contract says so), called through the C ABI binding (haag_vq._native)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _h(t):
    return t.detach().cpu().numpy()


def _codebook(rng, X, M, ksub, dups=True):
    """Centroids drawn from data rows + noise, with exact duplicates and near-duplicates."""
    n, d = X.shape
    dsub = d // M
    idx = rng.integers(0, n, size=ksub)
    C = X[idx].reshape(ksub, M, dsub).transpose(1, 0, 2).copy()
    C += rng.standard_normal(C.shape).astype(np.float32) * 0.05 * np.abs(C).mean()
    if dups and ksub >= 8:
        C[:, 5] = C[:, 3]                    # exact tie: canonical first index wins
        C[:, 7] = C[:, 6] * (1 + 1e-7)       # near tie
    return np.ascontiguousarray(C, dtype=np.float32)


PQ_SHAPES = [
    # n, d, M, nbits          path
    (1000, 1536, 16, 8),    # MFMA KS=6 (the headline shape)
    (777, 1024, 16, 8),     # MFMA KS=4, ragged n
    (513, 1536, 32, 8),     # MFMA KS=3 (OPQ32 shape)
    (300, 1024, 8, 8),      # wide filter KS=8 (dsub 128: K in two tile halves, 8 waves)
    (300, 1536, 8, 8),      # wide filter KS=12 (dsub 192: config #1's PQ8 at D=1536)
    (300, 1280, 8, 8),      # wide filter KS=10 (dsub 160, K halves of 5 steps, generic load layout)
    (300, 1120, 8, 8),      # wide filter KS=9 (dsub 140, padded K)
    (200, 1024, 4, 8),      # dsub 256 (M = 4 at D = 1024: the sweep's `--pq-subquantizers 4`)
    (150, 1536, 4, 8),      # dsub 384 (M = 4 at D = 1536)
    (200, 48, 6, 8),        # dsub 8, KS=1
    (257, 48, 12, 8),       # dsub 4
    (256, 16, 4, 4),        # nbits 4 (faiss bit stream)
    (100, 30, 10, 3),       # dsub 3, nbits 3 -> exact path + pack
    (64, 64, 8, 1),         # nbits 1
    (1, 1536, 16, 8),       # single row
]


@pytest.mark.parametrize("n,d,M,nbits", PQ_SHAPES)
def test_pq_encode_bit_exact(dev, oracle, n, d, M, nbits):
    from haag_vq import _native

    rng = np.random.default_rng(n * 7 + d + M)
    X = rng.standard_normal((n, d)).astype(np.float32)
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    Xtrain = rng.standard_normal((max(n, 1 << nbits), d)).astype(np.float32)
    Xtrain /= np.linalg.norm(Xtrain, axis=1, keepdims=True)
    C = _codebook(rng, Xtrain, M, 1 << nbits)
    # rows that sit exactly on centroids / between tied centroids
    if n > 10 and nbits >= 3:
        X[3] = C[:, 3].reshape(-1)
        X[4] = 0.5 * (C[:, 6] + C[:, 7]).reshape(-1)
    ref = oracle.pq_pack(oracle.pq_encode(X, C), nbits)
    Cd = _t(C, dev)
    prep = _native.pq_prepare(Cd, nbits)
    got = _h(_native.pq_encode(_t(X, dev), Cd, prep, nbits))
    np.testing.assert_array_equal(got, ref)
    got_exact = _h(_native.pq_encode(_t(X, dev), Cd, prep, nbits, exact=True))
    np.testing.assert_array_equal(got_exact, ref)
    got_legacy = _h(_native.pq_encode(_t(X, dev), Cd, prep, nbits, flags_extra=_native.MIVQ_PQ_LEGACY_MFMA))
    np.testing.assert_array_equal(got_legacy, ref)
    got_lexact = _h(_native.pq_encode(_t(X, dev), Cd, prep, nbits, exact=True,
                                      flags_extra=_native.MIVQ_PQ_LEGACY_EXACT))
    np.testing.assert_array_equal(got_lexact, ref)


@pytest.mark.parametrize("kind", ["gaussian", "clustered", "duplicates"])
def test_pq_encode_bit_exact_trained_codebooks(dev, oracle, kind):
    """Codebooks trained on the data (many near-ties), 20k rows, both MFMA kernels."""
    from haag_vq import _native
    from haag_vq.methods._kmeans import train_pq

    rng = np.random.default_rng(11)
    n, d, M = 20000, 1536, 16
    if kind == "gaussian":
        X = rng.standard_normal((n, d)).astype(np.float32)
    else:
        cen = rng.standard_normal((64, d)).astype(np.float32)
        X = cen[rng.integers(0, 64, n)] + 0.02 * rng.standard_normal((n, d)).astype(np.float32)
        if kind == "duplicates":
            X[1::2] = X[0::2]  # every row twice
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    Xd = _t(X, dev)
    C = train_pq(Xd, M, 8, niter=10)
    ref = oracle.pq_encode(X, _h(C))
    prep = _native.pq_prepare(C, 8)
    np.testing.assert_array_equal(_h(_native.pq_encode(Xd, C, prep, 8)), ref)
    np.testing.assert_array_equal(_h(_native.pq_encode(Xd, C, prep, 8, flags_extra=_native.MIVQ_PQ_LEGACY_MFMA)), ref)
    # the tiled exact kernel (register-blocked VALU GEMM, cross-lane argmin) on the same near-ties
    np.testing.assert_array_equal(_h(_native.pq_encode(Xd, C, prep, 8, exact=True)), ref)


@pytest.mark.parametrize("n,d,M", [(60_001, 1536, 8), (40_000, 1536, 12), (40_000, 1280, 8), (20_000, 1120, 8)])
def test_pq_encode_bit_exact_wide_subspaces(dev, oracle, n, d, M):
    """Wide subspaces on k-means codebooks (thousands of resolve items per workgroup): dsub 192,
    128, 160 run the K-halves filter (8 waves) and the resolve with rows in registers and the
    full-batch candidate lists; dsub 140 the 4-wave filter and the generic resolve."""
    from haag_vq import _native
    from haag_vq.methods._kmeans import train_pq

    rng = np.random.default_rng(d + M)
    X = rng.standard_normal((n, d)).astype(np.float32)
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    X[7] = X[3]  # duplicate rows
    Xd = _t(X, dev)
    C = train_pq(Xd[:16384], M, 8, niter=6)
    ref = oracle.pq_encode(X, _h(C))
    prep = _native.pq_prepare(C, 8)
    np.testing.assert_array_equal(_h(_native.pq_encode(Xd, C, prep, 8)), ref)


def test_pq_encode_bit_exact_config5_shape(dev, oracle):
    """D = 1024, M = 16 (dsub 64: the 16-wave filter specialisation of BASELINE config #5) on a
    k-means codebook, 120k rows (many row chunks per subspace, a ragged last chunk)."""
    from haag_vq import _native
    from haag_vq.methods._kmeans import train_pq

    rng = np.random.default_rng(5)
    n, d, M = 120_003, 1024, 16
    X = rng.standard_normal((n, d)).astype(np.float32)
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    Xd = _t(X, dev)
    C = train_pq(Xd[:20000], M, 8, niter=8)
    ref = oracle.pq_encode(X, _h(C))
    prep = _native.pq_prepare(C, 8)
    np.testing.assert_array_equal(_h(_native.pq_encode(Xd, C, prep, 8)), ref)


@pytest.mark.parametrize("nbits", [1, 2, 4, 8])
def test_extrabitq_kernels_match_reference_fixture(dev, golden_dir, nbits):
    """Device encode/decode of the reference's ExtendedRaBitQuantizer model state."""
    from haag_vq import _native

    e = np.load(golden_dir / "extrabitq_golden.npz")
    X = e["X"]
    tag = f"b{nbits}"
    c, P, lv = (_t(e[f"{tag}_{k}"], dev) for k in ("c", "P", "levels"))
    codes = _h(_native.extrabitq_encode(_t(X, dev), c, P, lv, nbits))
    ref = e[f"{tag}_codes"]
    ib = (X.shape[1] * nbits + 7) // 8
    # fp64 GEMM order differs from numpy: index bytes may differ only at level midpoints
    assert (codes[:, :ib] != ref[:, :ib]).mean() < 1e-3
    np.testing.assert_allclose(codes[:, ib:].copy().view(np.float32), ref[:, ib:].copy().view(np.float32), rtol=1e-6)
    rec = _h(_native.extrabitq_decode(_t(ref, dev), c, P, lv, nbits))
    np.testing.assert_allclose(rec, e[f"{tag}_recon"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n,d", [(1, 16), (77, 100), (300, 96), (257, 1536), (130, 3072)])
@pytest.mark.parametrize("transpose", [False, True])
def test_extrabitq_rotate_matches_fp64(dev, n, d, transpose):
    """mivq_extrabitq_rotate (fp64 MFMA GEMM, extended_rabitq.py:140,196) against a numpy fp64
    product: every element within a few ulps of sum |o_k P_kj| (fp64 accumulation, another
    summation order), ragged n and d past the 128 x 128 tiles and 16-wide K slices."""
    from haag_vq import _native

    rng = np.random.default_rng(n * 7 + d)
    o = rng.standard_normal((n, d))
    P, _ = np.linalg.qr(rng.standard_normal((d, d)))
    got = _h(_native.extrabitq_rotate(_t(o, dev), _t(P, dev), transpose))
    Pm = P.T if transpose else P
    ref = o @ Pm
    scale = np.abs(o) @ np.abs(Pm)
    assert np.all(np.abs(got - ref) <= 1e-14 * d * scale + 1e-300), float(np.max(np.abs(got - ref) / scale))


def _prep_offsets(M, dsub, ksub=256):
    """Byte offsets inside the mivq_pq_prepare buffer (mirror of PqPrepLayout, mivq_common.h)."""
    al = lambda v: (v + 255) // 256 * 256  # noqa: E731
    ks = (dsub + 15) // 16
    L, off = {}, 0
    for name, size in (("cn", 4 * M * ksub), ("ct", 4 * M * dsub * ksub), ("img", M * 8 * ks * 64 * 16),
                       ("hinit", 4 * M * ksub), ("bnd", 16 * M), ("spread", 8 * M),
                       ("pd", M * 256 * 256 * 8 if M <= 64 else 0), ("bnd2", 16 * M)):
        L[name] = off
        off = al(off + size)
    return L


@pytest.mark.parametrize("d,M", [(1536, 16), (1024, 16), (200, 4)])
def test_pq_prep_spreads_bound_the_image(dev, d, M):
    """The filter window rests on the measured spreads of the f16 image (pq_prep_spread_kernel):
    Dmax^2 / DDmax^2 (fp32 chains) within (dsub + 3) 2^-24 of the fp64 value, and every
    per-pair entry of pd an upper bound of the exact pair spread within 2e-5."""
    from haag_vq import _native

    rng = np.random.default_rng(11)
    dsub = d // M
    C = (rng.standard_normal((M, 256, dsub)) * rng.uniform(0.01, 3.0, (M, 1, 1))).astype(np.float32)
    prep = _native.pq_prepare(_t(C, dev), 8)
    torch.cuda.synchronize()
    raw = _h(prep)
    L = _prep_offsets(M, dsub)
    spread = raw[L["spread"]:L["spread"] + 8 * M].view(np.float32).reshape(M, 2)
    pd = raw[L["pd"]:L["pd"] + M * 256 * 256 * 8].view(np.float32).reshape(M, 256, 256, 2)
    rel = (dsub + 3) * 2.0 ** -24 * 1.01
    for m in range(M):
        e = int(np.ceil(np.log2(np.abs(C[m]).max())))
        t = (C[m] * np.float32(2.0 ** (14 - e))).astype(np.float32)
        h = t.astype(np.float16).astype(np.float32)
        r = (h - t).astype(np.float64)
        h = h.astype(np.float64)
        d1 = ((h[:, None, :] - h[None, :, :]) ** 2).sum(-1)
        d2 = ((r[:, None, :] - r[None, :, :]) ** 2).sum(-1)
        for got, ref in ((spread[m, 0], d1.max()), (spread[m, 1], d2.max())):
            assert abs(float(got) - ref) <= rel * ref + 1e-30, (m, got, ref)
        for k, ref in ((0, np.sqrt(d1)), (1, np.sqrt(d2))):
            got = pd[m, :, :, k].astype(np.float64)
            assert (got >= ref * (1 - 1e-7)).all() and (got <= ref * (1 + 2e-5) + 1e-30).all(), m


def test_pq_encode_extreme_rows_fall_back_exactly(dev, oracle):
    """fp16 overflow (huge rows), NaN rows and zero rows take the exact fallback."""
    from haag_vq import _native

    rng = np.random.default_rng(5)
    n, d, M = 300, 1536, 16
    X = rng.standard_normal((n, d)).astype(np.float32)
    C = _codebook(rng, X, M, 256)
    X[10] *= 1e6
    X[11] = 0.0
    X[12, :5] = np.nan
    X[13] *= 1e-12
    ref = oracle.pq_encode(X, C)
    Cd = _t(C, dev)
    prep = _native.pq_prepare(Cd, 8)
    got = _h(_native.pq_encode(_t(X, dev), Cd, prep, 8))
    np.testing.assert_array_equal(got, ref)


def test_pq_encode_matches_fp64_on_clear_cases(dev, oracle):
    from haag_vq import _native

    rng = np.random.default_rng(9)
    X = rng.standard_normal((400, 1536)).astype(np.float32)
    C = _codebook(rng, X, 16, 256, dups=False)
    codes64, gap = oracle.pq_encode_fp64(X, C)
    Cd = _t(C, dev)
    got = _h(_native.pq_encode(_t(X, dev), Cd, _native.pq_prepare(Cd, 8), 8))
    clear = gap > 1e-5
    assert clear.mean() > 0.9
    np.testing.assert_array_equal(got[clear], codes64[clear])


@pytest.mark.parametrize("n,d,M,nbits", [(300, 1536, 16, 8), (256, 16, 4, 4), (100, 30, 10, 3)])
def test_pq_decode_bit_exact(dev, oracle, n, d, M, nbits):
    from haag_vq import _native

    rng = np.random.default_rng(1)
    C = rng.standard_normal((M, 1 << nbits, d // M)).astype(np.float32)
    u8 = rng.integers(0, 1 << nbits, size=(n, M)).astype(np.uint8)
    packed = oracle.pq_pack(u8, nbits)
    ref = oracle.pq_decode(u8, C)
    got = _h(_native.pq_decode(_t(packed, dev), _t(C, dev), nbits))
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(_h(_native.pq_unpack(_t(packed, dev), M, nbits)), u8)


def test_pq_encode_empty(dev):
    from haag_vq import _native

    C = torch.zeros((16, 256, 96), device=dev)
    prep = _native.pq_prepare(C, 8)
    out = _native.pq_encode(torch.zeros((0, 1536), device=dev), C, prep, 8)
    assert tuple(out.shape) == (0, 16)


def test_pq_errors(dev):
    from haag_vq import _native

    C = torch.zeros((16, 256, 96), device=dev)
    with pytest.raises(ValueError):
        _native.pq_encode(torch.zeros((4, 1000), device=dev), C, _native.pq_prepare(C, 8), 8)
    with pytest.raises(ValueError):
        _native.pq_prepare(torch.zeros((16, 100, 96), device=dev), 8)


def test_sq_golden_bit_exact(dev, golden_dir):
    from haag_vq import _native

    g = np.load(golden_dir / "sq_golden.npz")
    for tag in g["cases"]:
        tag = str(tag)
        X, lo, hi, codes, recon = (g[f"{tag}_{k}"] for k in ("X", "lo", "hi", "codes", "recon"))
        bits = int(tag.split("_b")[1])
        den = (hi - lo) + 1e-8
        c = _h(_native.sq_encode(_t(X, dev), _t(lo, dev), _t(den, dev), bits))
        if bits == 16:
            c = c.view(np.uint16)
        np.testing.assert_array_equal(c, codes, err_msg=tag)
        ct = _t(codes.view(np.int16) if bits == 16 else codes, dev)
        r = _h(_native.sq_decode(ct, X.shape[1], _t(lo, dev), _t(den, dev), bits))
        assert r.dtype == recon.dtype, tag
        np.testing.assert_array_equal(r.view(np.uint8), recon.view(np.uint8), err_msg=tag)


@pytest.mark.parametrize("bits", [4, 8, 16])
def test_sq_vector_path_equals_generic(dev, bits):
    """The aligned f32 encode (column-stationary kernel) against the generic kernel (taken for
    d % 8 != 0): the first d columns of X and of X with one extra column go through the two
    paths with the same lo / den, and their codes must be identical, over wide magnitudes,
    values on both sides of the data range, non-finite entries and extreme den values."""
    from haag_vq import _native

    n, d = 200_000, 64
    g = torch.Generator(device=dev).manual_seed(bits)
    scale = torch.logspace(-30, 30, d, device=dev)
    X = torch.randn((n, d), device=dev, generator=g) * scale
    X[::97, 5] = float("nan")
    X[::89, 6] = float("inf")
    lo = X.nan_to_num(posinf=0.0).amin(0) * 0.9
    hi = X.nan_to_num(posinf=0.0).amax(0) * 0.9  # values beyond both ends of the range
    den = (hi - lo) + 1e-8
    den[7] = 3.0e36   # beyond the reciprocal range: that group divides
    den[8] = 1.0e-35
    Xp = torch.cat([X, torch.zeros((n, 1), device=dev)], 1).contiguous()
    lop = torch.cat([lo, lo[:1]]).contiguous()
    denp = torch.cat([den, den[:1]]).contiguous()
    a = _native.sq_encode(X.contiguous(), lo.contiguous(), den.contiguous(), bits)
    b = _native.sq_encode(Xp, lop, denp, bits)
    if bits == 4:
        np.testing.assert_array_equal(_h(a), _h(b)[:, : d // 2])
    else:
        np.testing.assert_array_equal(_h(a), _h(b)[:, :d])


@pytest.mark.parametrize("bits", [8, 16])
def test_sq_vector_path_division_at_rounding_boundaries(dev, bits):
    """The vector path divides through a correctly rounded reciprocal plus one residual
    correction (sq.hip: div_rn_rcp); the generic kernel uses the IEEE division.  Elements are
    placed so that (x - lo) / den * L lands within a few ulps of a rounding boundary k + 1/2,
    where a quotient one ulp off flips the code: both paths must agree on every element, over
    den magnitudes 2^-60..2^60 and both signs of x - lo."""
    from haag_vq import _native

    n, d = 100_000, 64
    L = (1 << bits) - 1
    g = torch.Generator(device=dev).manual_seed(17 + bits)
    den = torch.logspace(-18, 18, d, device=dev, dtype=torch.float64)
    lo = torch.randn((d,), device=dev, generator=g, dtype=torch.float64) * den
    k = torch.randint(0, L, (n, d), device=dev, generator=g).double()
    t = (k + 0.5) / L + torch.randint(-3, 4, (n, d), device=dev, generator=g).double() * 2.0 ** -24 / L
    X = (lo + den * t).float()
    X[1::2] = (lo - den * t[1::2]).float()  # negative quotients (clipped by the cast)
    lo32, den32 = lo.float().contiguous(), den.float().contiguous()
    Xp = torch.cat([X, torch.zeros((n, 1), device=dev)], 1).contiguous()
    a = _native.sq_encode(X.contiguous(), lo32, den32, bits)
    b = _native.sq_encode(Xp, torch.cat([lo32, lo32[:1]]).contiguous(), torch.cat([den32, den32[:1]]).contiguous(),
                          bits)
    np.testing.assert_array_equal(_h(a), _h(b)[:, :d])


@pytest.mark.parametrize("n,d", [(500, 1024), (333, 3072), (77, 37)])
@pytest.mark.parametrize("metric", [1, 0])
def test_rabitq_parity(dev, oracle, n, d, metric):
    from haag_vq import _native

    rng = np.random.default_rng(d)
    X = rng.standard_normal((n, d)).astype(np.float32)
    X[0] = 0.0  # degenerate row (epsilon guards)
    ref = oracle.rabitq_encode(X, metric=metric)
    got = _h(_native.rabitq_encode(_t(X, dev), None, metric))
    nb = (d + 7) // 8
    np.testing.assert_array_equal(got[:, :nb], ref[:, :nb])
    f_ref = ref[:, nb:].copy().view(np.float32)
    f_got = got[:, nb:].copy().view(np.float32)
    np.testing.assert_allclose(f_got, f_ref, rtol=1e-5, atol=1e-5 * np.abs(f_ref).max())
    rec = _h(_native.rabitq_decode(_t(got, dev), d, None))
    np.testing.assert_array_equal(rec, oracle.rabitq_decode(got, d))  # same code row -> same floats


@pytest.mark.parametrize("n,d", [(300, 1024), (129, 1536), (257, 3072), (65, 2048), (40, 520)])
def test_rabitq_parity_with_centroid(dev, oracle, n, d):
    """The centroid path of every rabitq_encode kernel (the batched-load kernel at d % 512 == 0
    with 2 / 3 / 6 / 4 bytes per lane, the generic kernel at d = 520): sign bits exact, factors
    within the 1e-5 contract of the sequential restatement."""
    from haag_vq import _native

    rng = np.random.default_rng(d + 1)
    X = rng.standard_normal((n, d)).astype(np.float32)
    c = (0.1 * rng.standard_normal(d)).astype(np.float32)
    X[1] = c  # residual exactly zero
    ref = oracle.rabitq_encode(X, c, metric=1)
    got = _h(_native.rabitq_encode(_t(X, dev), _t(c, dev), 1))
    nb = (d + 7) // 8
    np.testing.assert_array_equal(got[:, :nb], ref[:, :nb])
    f_ref = ref[:, nb:].copy().view(np.float32)
    f_got = got[:, nb:].copy().view(np.float32)
    np.testing.assert_allclose(f_got, f_ref, rtol=1e-5, atol=1e-5 * np.abs(f_ref).max())


@pytest.mark.parametrize("nq,n,d,M,nbits,k", [
    (37, 5000, 1536, 16, 8, 10),    # LUT: compile-time dsub 96
    (9, 3000, 1536, 32, 8, 100),    # dsub 48
    (11, 2000, 1024, 16, 8, 10),    # dsub 64
    (13, 700, 256, 2, 8, 10),       # packed LUT kernel, run-time dsub (128)
    (16, 1000, 64, 8, 4, 7),
    (5, 200, 48, 6, 8, 256),
    (3, 5, 64, 8, 8, 10),   # fewer rows than k: sentinel slots
])
@pytest.mark.parametrize("metric", [1, 0])
def test_adc_bit_exact(dev, oracle, nq, n, d, M, nbits, k, metric):
    from haag_vq import _native

    rng = np.random.default_rng(nq + n)
    C = rng.standard_normal((M, 1 << nbits, d // M)).astype(np.float32)
    Q = rng.standard_normal((nq, d)).astype(np.float32)
    u8 = rng.integers(0, 1 << nbits, size=(n, M)).astype(np.uint8)
    u8[1] = u8[0]  # duplicate rows: equal distances, id tie-break
    lut_ref = oracle.adc_lut(Q, C, metric)
    lut = _native.adc_lut(_t(Q, dev), _t(C, dev), nbits, metric)
    np.testing.assert_array_equal(_h(lut), lut_ref)
    d_ref, i_ref = oracle.adc_search(lut_ref, u8, k)
    dd, ii = _native.adc_search(lut, _t(u8, dev), k, nbits)
    np.testing.assert_array_equal(_h(dd), d_ref)
    np.testing.assert_array_equal(_h(ii).view(np.uint32), i_ref)


@pytest.mark.parametrize("offset", [1, 2, 3])
def test_adc_lut_misaligned_centroids(dev, oracle, offset):
    """A centroid tensor that starts off a 16-B boundary (a view with storage_offset % 4 != 0,
    or a C-API caller's pointer): the LUT kernel takes its dword path instead of 16-B loads."""
    from haag_vq import _native

    rng = np.random.default_rng(40 + offset)
    M, dsub, nq = 16, 96, 40
    C = rng.standard_normal((M, 256, dsub)).astype(np.float32)
    Q = rng.standard_normal((nq, M * dsub)).astype(np.float32)
    flat = torch.zeros(C.size + offset, dtype=torch.float32, device=dev)
    flat[offset:] = _t(C.reshape(-1), dev)
    Cv = flat[offset:].view(M, 256, dsub)
    assert Cv.data_ptr() % 16 != 0
    for metric in (1, 0):
        np.testing.assert_array_equal(_h(_native.adc_lut(_t(Q, dev), Cv, 8, metric)), oracle.adc_lut(Q, C, metric))


@pytest.mark.parametrize("nq,n,d,k", [
    (20, 3000, 1024, 10), (7, 500, 37, 100), (4, 3, 16, 5),    # streaming scan
    (100, 20000, 96, 10),                                         # tiled, one chunk, 5 segments
    (4100, 40000, 16, 10),                                        # tiled, 3 chunks + running merge
    (64, 5000, 30, 100),                                          # tiled, d % 4 != 0
    (16, 4096, 1536, 256),                                        # tiled, k = 256
])
@pytest.mark.parametrize("metric", [1, 0])
def test_flat_search_bit_exact(dev, oracle, nq, n, d, k, metric):
    from haag_vq import _native

    rng = np.random.default_rng(d)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((nq, d)).astype(np.float32)
    if n > 100:
        X[n - 1] = X[3]      # exact duplicate across segments / chunks: smaller id first
        X[n // 2] = X[3]
    d_ref, i_ref = oracle.flat_search(Q, X, k, metric)
    dd, ii = _native.flat_search(_t(Q, dev), _t(X, dev), k, metric)
    np.testing.assert_array_equal(_h(dd), d_ref)
    np.testing.assert_array_equal(_h(ii).view(np.uint32), i_ref)


def test_sharded_adc_merge_equals_single(dev, oracle):
    """Row shards searched with id offsets and merged == one search (multi-GPU contract)."""
    from haag_vq import _native

    rng = np.random.default_rng(3)
    nq, n, M, k = 11, 4000, 16, 10
    C = rng.standard_normal((M, 256, 8)).astype(np.float32)
    Q = rng.standard_normal((nq, M * 8)).astype(np.float32)
    u8 = rng.integers(0, 256, size=(n, M)).astype(np.uint8)
    lut = _native.adc_lut(_t(Q, dev), _t(C, dev), 8)
    full_d, full_i = _native.adc_search(lut, _t(u8, dev), k, 8)
    for parts in (2, 3, 8):
        bounds = np.linspace(0, n, parts + 1).astype(int)
        ds, is_ = [], []
        for a, b in zip(bounds[:-1], bounds[1:]):
            d_, i_ = _native.adc_search(lut, _t(u8[a:b], dev), k, 8, id_offset=int(a))
            ds.append(d_)
            is_.append(i_)
        md, mi = _native.topk_merge(torch.stack(ds).contiguous(), torch.stack(is_).contiguous(), k)
        np.testing.assert_array_equal(_h(md), _h(full_d))
        np.testing.assert_array_equal(_h(mi), _h(full_i))


def test_opq_rotate(dev):
    from haag_vq import _native

    rng = np.random.default_rng(4)
    for n, d in ((1000, 1536), (130, 100), (7, 48)):
        X = rng.standard_normal((n, d)).astype(np.float32)
        A = np.linalg.qr(rng.standard_normal((d, d)))[0].astype(np.float32)
        y = _h(_native.opq_rotate(_t(X, dev), _t(A, dev), False))
        ref = X.astype(np.float64) @ A.astype(np.float64).T
        tol = 1e-5 * np.linalg.norm(X, axis=1, keepdims=True)
        assert np.all(np.abs(y - ref) <= tol + 1e-30)
        back = _h(_native.opq_rotate(_t(y, dev), _t(A, dev), True))
        ref2 = y.astype(np.float64) @ A.astype(np.float64)
        assert np.all(np.abs(back - ref2) <= tol + 1e-30)


@pytest.mark.parametrize("n,M,ksub,dsub", [(5000, 4, 16, 8), (600, 2, 8, 384), (300, 1, 4, 1536)])
def test_kmeans_update_deterministic(dev, n, M, ksub, dsub):
    """Centroid update: ascending-row sums, empty clusters keep their value; dsub past 256
    (M = 4 at D = 1536 is dsub 384, the reference sweep's `--pq-subquantizers 4`)."""
    from haag_vq import _native

    rng = np.random.default_rng(8)
    X = rng.standard_normal((n, M * dsub)).astype(np.float32)
    assign = rng.integers(0, ksub - 1, size=(n, M)).astype(np.uint8)  # last cluster empty
    C0 = rng.standard_normal((M, ksub, dsub)).astype(np.float32)
    Cd = _t(C0, dev)
    counts = torch.empty((M, ksub), dtype=torch.int32, device=dev)
    _native.kmeans_update(_t(X, dev), _t(assign, dev), Cd, counts)
    C = _h(Cd)
    cnt = _h(counts)
    Xs = X.reshape(n, M, dsub)
    for m in range(M):
        for k in range(ksub):
            sel = assign[:, m] == k
            assert cnt[m, k] == sel.sum()
            if sel.sum():
                # ascending-row sequential f32 sum, then one division
                s = np.zeros(dsub, np.float32)
                for row in np.nonzero(sel)[0]:
                    s = (s + Xs[row, m]).astype(np.float32)
                np.testing.assert_array_equal(C[m, k], (s / np.float32(sel.sum())).astype(np.float32))
            else:
                np.testing.assert_array_equal(C[m, k], C0[m, k])


@pytest.mark.parametrize("nq,n,d,qb,k", [
    (37, 3000, 1536, 4, 10),    # MFMA path, the RaBitQIndex default qb
    (40, 1000, 256, 8, 17),     # qb = 8: int8 offset 128
    (33, 777, 96, 1, 5),        # qb = 1, ragged tiles
    (9, 500, 100, 4, 10),       # d % 32 != 0: generic kernel
    (5, 300, 64, 0, 8),         # qb = 0: float estimator (generic kernel)
    (3, 5, 64, 4, 10),          # fewer codes than k: sentinel slots
    (16500, 8500, 32, 4, 3),    # three column chunks of the tiled top-k
    (150, 3000, 512, 4, 10),    # multi-query kernel, 128 queries per workgroup, ragged last block
    (1000, 20000, 512, 4, 10),  # persistent multi-query kernel: each workgroup walks several code groups
])
@pytest.mark.parametrize("metric", [1, 0])
def test_rabitq_search_bit_exact(dev, oracle, nq, n, d, qb, k, metric):
    from haag_vq import _native

    rng = np.random.default_rng(nq + n + d + qb)
    X = rng.standard_normal((n, d)).astype(np.float32)
    X[n // 2] = X[n // 3]  # duplicate code: tie broken by the smaller id
    Q = rng.standard_normal((nq, d)).astype(np.float32)
    Q[0] = 0.25  # constant query residual -> delta = 0 guard
    c = X.mean(0).astype(np.float32)
    cd = _t(c, dev)
    codes = _native.rabitq_encode(_t(X, dev), cd, metric)
    kd, ki = _native.rabitq_search(codes, d, cd, _t(Q, dev), qb, metric, k)
    keys = oracle.rabitq_est(_h(codes), d, Q, c, qb, metric)
    rd, ri = oracle.topk_rows(keys, k)
    np.testing.assert_array_equal(_h(ki).view(np.uint32), ri)
    np.testing.assert_array_equal(_h(kd), rd)


@pytest.mark.parametrize("k,metric,order", [
    (10, 1, "worst"),     # every later code beats every earlier one for query 0: all pass the screen
    (100, 1, "random"),   # two-register lists
    (256, 0, "worst"),    # k = 256, inner product
    (10, 0, "random"),
])
def test_rabitq_search_screened_blocks(dev, oracle, k, metric, order):
    """The screened search of the multi-query kernel (d % 512 == 0): a dense first block (two
    column chunks of the tiled top-k at nq = 16500), then five screened blocks whose keys are appended
    only when they beat the query's running k-th element, merged in place.  Codes ordered so
    that query 0 finds a better code at every later position (its lists hold whole blocks),
    exact duplicates of first-block codes in later blocks (ties must keep the smaller id), a
    ragged last query block; checked against the oracle on a subset of the queries."""
    from haag_vq import _native

    rng = np.random.default_rng(k + metric)
    nq, n, d = 16500, 40000, 512
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((nq, d)).astype(np.float32)
    c = X.mean(0).astype(np.float32)
    cd = _t(c, dev)
    codes = _h(_native.rabitq_encode(_t(X, dev), cd, metric))
    if order == "worst":
        keys0 = oracle.rabitq_est(codes, d, Q[:1], c, 4, metric)[0]
        codes = codes[np.argsort(-keys0, kind="stable")]
    dup_src = rng.choice(8000, 300, replace=False)
    dup_dst = 8192 + rng.choice(n - 8192, 300, replace=False)
    codes[dup_dst] = codes[dup_src]
    codes = np.ascontiguousarray(codes)
    kd, ki = _native.rabitq_search(_t(codes, dev), d, cd, _t(Q, dev), 4, metric, k)
    sub = np.r_[0, 1, 31, 32, 127, 128, 2049, rng.choice(nq, 24, replace=False), nq - 4, nq - 1]
    keys = oracle.rabitq_est(codes, d, Q[sub], c, 4, metric)
    rd, ri = oracle.topk_rows(keys, k)
    np.testing.assert_array_equal(_h(ki)[sub].view(np.uint32), ri)
    np.testing.assert_array_equal(_h(kd)[sub], rd)


@pytest.mark.parametrize("d", [96, 192])
def test_pq_encode_slice_boundary_wide_shapes(dev, oracle, d):
    """the slicing of large calls (2^20-row slices since round 5) at the shapes it was
    tuned for — dsub 96 (KS 6, the D96 wave count) and dsub 192 (KS 12, K-halves filter) with
    M = 1 — rows on both sides of the boundaries and the ragged last slice (1001 rows: the
    generic code transpose) vs the oracle."""
    from haag_vq import _native

    rng = np.random.default_rng(d)
    n = (1 << 21) + 1001
    Xd = torch.randn((n, d), device=dev, generator=torch.Generator(device=dev).manual_seed(d))
    X0 = _h(Xd[:4096])
    C = _codebook(rng, X0, 1, 256)
    Cd = _t(C, dev)
    got = _h(_native.pq_encode(Xd, Cd, _native.pq_prepare(Cd, 8), 8))
    for lo, hi in ((0, 1500), ((1 << 20) - 2500, (1 << 20) + 2500), ((1 << 21) - 2500, n)):
        np.testing.assert_array_equal(got[lo:hi], oracle.pq_encode(_h(Xd[lo:hi]), C))


def test_pq_encode_slices_large_calls(dev, oracle):
    """Calls above 2^20 rows run as 2^20-row slices: rows on both sides of slice boundaries
    (2^20, 2^21, 2^22) and in the ragged last slice equal the oracle."""
    from haag_vq import _native

    rng = np.random.default_rng(21)
    n, d, M = (1 << 22) + 1001, 64, 16
    X = rng.standard_normal((n, d), dtype=np.float32)
    C = _codebook(rng, X[:4096], M, 256)
    Cd = _t(C, dev)
    got = _h(_native.pq_encode(_t(X, dev), Cd, _native.pq_prepare(Cd, 8), 8))
    for lo, hi in ((0, 2000), ((1 << 20) - 3000, (1 << 20) + 3000), ((1 << 21) - 3000, (1 << 21) + 3000),
                   ((1 << 22) - 2000, n)):
        np.testing.assert_array_equal(got[lo:hi], oracle.pq_encode(np.ascontiguousarray(X[lo:hi]), C))
