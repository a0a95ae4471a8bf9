"""Reference-generated fixtures at the BASELINE widths (tests/golden/make_golden.py `wide`).

SQ 4/8/16 bits at D = 1024 and 3072 (fp32 and fp64 rows; BASELINE configs[3] is SQ-8 on
1M x 3072) and Extended RaBitQ at D = 1024 and (round 5) D = 3072 -- the width of bench.py's
Extended RaBitQ leg --, produced by importing the reference's
ScalarQuantizer (scalar_quantization.py:52-90) and ExtendedRaBitQuantizer
(extended_rabitq.py:125-199) in the build container.  The input rows are regenerated from the
stored seeds (their sha256 is checked first, so generator drift fails loudly instead of
comparing against the wrong data); full outputs are compared through sha256 digests, the first
rows verbatim.

CPU tests pin the oracle to these fixtures; `-m gpu` tests run the HIP kernels
(sq_encode_f32_vec_kernel / sq_encode_f64 / sq_decode, the mivq_extrabitq_* path) on them.
"""

import hashlib
import importlib.util

import numpy as np
import pytest
import torch


def _sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def mk(golden_dir):
    spec = importlib.util.spec_from_file_location("make_golden", golden_dir / "make_golden.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)  # defines the input generators; imports nothing of the reference
    return m


@pytest.fixture(scope="module")
def sqw(golden_dir):
    return np.load(golden_dir / "sq_golden_wide.npz")


@pytest.fixture(scope="module")
def erqw(golden_dir):
    return np.load(golden_dir / "extrabitq_golden_wide.npz")


@pytest.fixture(scope="module")
def erq3k(golden_dir):
    return np.load(golden_dir / "extrabitq_golden_3072.npz")


def _sq_case(g, mk, tag):
    dtype = np.float64 if tag.startswith("float64") else np.float32
    d = int(tag.split("_d")[1].split("_")[0])
    bits = int(tag.split("_b")[1])
    X = mk.sq_wide_input(dtype, d, int(g[f"{tag}_seed"]))
    assert _sha(X) == str(g[f"{tag}_X_sha"]), f"{tag}: regenerated input differs from the fixture's"
    lo, hi = g[f"{tag}_lo"], g[f"{tag}_hi"]
    return X, lo, hi, (hi - lo) + 1e-8, bits


def _check_sq(g, tag, codes, recon):
    cd = np.dtype(str(g[f"{tag}_codes_dtype"]))
    codes = codes.view(cd) if codes.dtype != cd else codes
    np.testing.assert_array_equal(codes[:4], g[f"{tag}_codes_head"], err_msg=tag)
    assert _sha(codes) == str(g[f"{tag}_codes_sha"]), tag
    assert recon.dtype == np.dtype(str(g[f"{tag}_recon_dtype"])), tag
    np.testing.assert_array_equal(recon[:4].view(np.uint8), g[f"{tag}_recon_head"].view(np.uint8), err_msg=tag)
    assert _sha(recon) == str(g[f"{tag}_recon_sha"]), tag


def test_sq_wide_oracle_matches_reference(oracle, sqw, mk):
    assert len(sqw["cases"]) == 12
    for tag in map(str, sqw["cases"]):
        X, lo, hi, den, bits = _sq_case(sqw, mk, tag)
        c = oracle.sq_encode(X, lo, den, bits)
        _check_sq(sqw, tag, c, oracle.sq_decode(c, X.shape[1], lo, den, bits))


def _erq_unpack(cb, D, nb):
    ib = (D * nb + 7) // 8
    bits = np.unpackbits(cb[:, :ib], axis=1)[:, :D * nb].reshape(len(cb), D, nb)
    return (bits.astype(np.int64) << np.arange(nb - 1, -1, -1)).sum(-1)


def _check_P(erqw, tag, P):
    """The regenerated rotation equals the fixture's to rounding (numpy's QR is bit-identical
    only on the same CPU: the sha is compared where it can be, the samples everywhere; the
    tolerances grow with D as the QR's rounding does)."""
    f = P.shape[0] / 1024
    np.testing.assert_allclose(P[:8], erqw[f"{tag}_P_head"], rtol=0, atol=1e-13 * f)
    np.testing.assert_allclose(P.sum(axis=0), erqw[f"{tag}_P_colsum"], rtol=0, atol=1e-12 * f ** 1.5)
    return _sha(P) == str(erqw[f"{tag}_P_sha"])


def _assert_ties_only(got, ref, X, c, P, lv, nbits, max_frac=1e-3):
    """Index mismatches only where s sits on a level midpoint (fp64 rounding), one level apart."""
    N, D = X.shape
    gi, ri = _erq_unpack(got, D, nbits), _erq_unpack(ref, D, nbits)
    bad = np.argwhere(gi != ri)
    r = X.astype(np.float64) - c
    s = (r / np.maximum(np.linalg.norm(r, axis=1), 1e-12)[:, None] @ P) * np.sqrt(D)
    mids = 0.5 * (lv[:-1] + lv[1:])
    for i, j in bad:
        assert np.min(np.abs(mids - s[i, j])) <= 1e-12 * max(1.0, abs(s[i, j])), (i, j)
        assert abs(int(gi[i, j]) - int(ri[i, j])) == 1
    assert len(bad) <= max_frac * N * D
    return bad


def test_extrabitq_wide_oracle_matches_reference(oracle, erqw, mk):
    X = mk.erq_wide_input()
    assert _sha(X) == str(erqw["X_sha"])
    for tag in map(str, erqw["cases"]):
        b = int(tag[1:])
        c, P, lv = oracle.extrabitq_fit(X, b)
        np.testing.assert_array_equal(c, erqw[f"{tag}_c"])
        same_P = _check_P(erqw, tag, P)
        np.testing.assert_array_equal(lv, erqw[f"{tag}_levels"])
        codes = oracle.extrabitq_encode(X, c, P, lv, b)
        if same_P:  # the generating machine: bit-exact
            np.testing.assert_array_equal(codes, erqw[f"{tag}_codes"])
            np.testing.assert_array_equal(oracle.extrabitq_decode(codes[:32], c, P, lv, b), erqw[f"{tag}_recon_head"])
        else:
            _assert_ties_only(codes, erqw[f"{tag}_codes"], X, c, P, lv, b)


def test_extrabitq_3072_oracle_matches_reference(oracle, erq3k, mk):
    """D = 3072 (bits 1 and 4, 64 rows): the oracle reproduces the reference's fit, codes and
    decode bit for bit where this CPU's QR reproduces the fixture's P (the generating machine);
    elsewhere the codes may differ only at proven level-midpoint ties."""
    X = mk.erq_3072_input()
    assert _sha(X) == str(erq3k["X_sha"])
    for tag in map(str, erq3k["cases"]):
        b = int(tag[1:])
        c, P, lv = oracle.extrabitq_fit(X, b)
        np.testing.assert_array_equal(c, erq3k[f"{tag}_c"])
        same_P = _check_P(erq3k, tag, P)
        np.testing.assert_array_equal(lv, erq3k[f"{tag}_levels"])
        codes = oracle.extrabitq_encode(X, c, P, lv, b)
        if same_P:
            np.testing.assert_array_equal(codes, erq3k[f"{tag}_codes"])
            np.testing.assert_array_equal(oracle.extrabitq_decode(codes[:32], c, P, lv, b), erq3k[f"{tag}_recon_head"])
        else:
            _assert_ties_only(codes, erq3k[f"{tag}_codes"], X, c, P, lv, b)


# ------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_sq_wide_gpu_bit_exact(dev, sqw, mk):
    """sq_encode at D = 1024 / 3072 (the f32 rows take the vector kernel, d % 8 == 0) and
    sq_decode: codes and reconstructions byte-identical to the reference's, all 256 rows."""
    from haag_vq import _native

    for tag in map(str, sqw["cases"]):
        X, lo, hi, den, bits = _sq_case(sqw, mk, tag)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        c = _native.sq_encode(t(X), t(lo), t(den), bits).cpu().numpy()
        cref = c.view(np.uint16) if bits == 16 else c
        ct = t(cref.view(np.int16) if bits == 16 else cref)
        r = _native.sq_decode(ct, X.shape[1], t(lo), t(den), bits).cpu().numpy()
        _check_sq(sqw, tag, cref, r)


@pytest.mark.gpu
@pytest.mark.parametrize("nbits", [1, 2, 4, 8])
def test_extrabitq_wide_gpu(dev, erqw, mk, oracle, nbits):
    """D = 1024: GPU indices equal the reference's except level-midpoint ties (fp64 summation
    order, as tests/test_pinning_gpu.py proves at D = 64), norms / t factors within 1e-6
    relative, and the GPU decode of the REFERENCE codes within 1e-6 of the reference's decode."""
    from haag_vq import _native

    X = mk.erq_wide_input()
    tag = f"b{nbits}"
    c, P, lv = oracle.extrabitq_fit(X, nbits)
    _check_P(erqw, tag, P)  # this machine's QR of the seeded matrix = the fixture's to rounding
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    ref = erqw[f"{tag}_codes"]
    got = _native.extrabitq_encode(t(X), t(c), t(P), t(lv), nbits).cpu().numpy()
    N, D = X.shape
    bad = _assert_ties_only(got, ref, X, c, P, lv, nbits)
    ib = (D * nbits + 7) // 8
    fg, fr = got[:, ib:].copy().view(np.float32), ref[:, ib:].copy().view(np.float32)
    ok_rows = np.setdiff1d(np.arange(N), bad[:, 0])  # t depends on every index of its row
    np.testing.assert_allclose(fg[ok_rows], fr[ok_rows], rtol=1e-6, atol=0)
    np.testing.assert_allclose(fg[:, 0], fr[:, 0], rtol=1e-6, atol=0)  # the norm never does
    dec = _native.extrabitq_decode(t(ref[:32]), t(c), t(P), t(lv), nbits).cpu().numpy()
    head = erqw[f"{tag}_recon_head"]
    np.testing.assert_allclose(dec, head, rtol=1e-6, atol=1e-6 * np.abs(head).max())


@pytest.mark.gpu
@pytest.mark.parametrize("nbits", [1, 4])
def test_extrabitq_3072_gpu(dev, erq3k, mk, oracle, nbits):
    """D = 3072: the HIP path against the reference's codes where this machine's QR gives the
    fixture's P bit for bit, otherwise against the oracle on this machine's P (the CPU test
    pins the oracle to the reference); indices equal except level-midpoint ties, norms / t
    factors within 1e-6, the GPU decode of the reference codes within 1e-6 of the reference's."""
    from haag_vq import _native

    X = mk.erq_3072_input()
    tag = f"b{nbits}"
    c, P, lv = oracle.extrabitq_fit(X, nbits)
    same_P = _check_P(erq3k, tag, P)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    ref = erq3k[f"{tag}_codes"] if same_P else oracle.extrabitq_encode(X, c, P, lv, nbits)
    got = _native.extrabitq_encode(t(X), t(c), t(P), t(lv), nbits).cpu().numpy()
    N, D = X.shape
    bad = _assert_ties_only(got, ref, X, c, P, lv, nbits)
    ib = (D * nbits + 7) // 8
    fg, fr = got[:, ib:].copy().view(np.float32), ref[:, ib:].copy().view(np.float32)
    ok_rows = np.setdiff1d(np.arange(N), bad[:, 0])
    np.testing.assert_allclose(fg[ok_rows], fr[ok_rows], rtol=1e-6, atol=0)
    np.testing.assert_allclose(fg[:, 0], fr[:, 0], rtol=1e-6, atol=0)
    head = erq3k[f"{tag}_recon_head"] if same_P else oracle.extrabitq_decode(ref[:32], c, P, lv, nbits)
    dec = _native.extrabitq_decode(t(ref[:32]), t(c), t(P), t(lv), nbits).cpu().numpy()
    np.testing.assert_allclose(dec, head, rtol=1e-6, atol=1e-6 * np.abs(head).max())
