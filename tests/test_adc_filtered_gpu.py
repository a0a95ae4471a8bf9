"""The filtered ADC search (adc.hip: integer-LUT scan + exact fp32 re-rank + certificate, the
fp32 scan re-run on uncertified queries) returns exactly the canonical top-k of
FlatQuantizedIndex.search_with_scores' ADC counterpart
(/root/reference/src/haag_vq/methods/search/flat_quantized_index.py:45-76): the oracle's
answer and the library's fp32-only scan (flag MIVQ_ADC_FORCE_EXACT), bit for bit, on inputs built to
defeat the filter (every row the same code, a handful of distinct rows, near-equal LUT
entries, non-finite LUTs) and on the shape edges (k = 1 / 32 on the filtered path, k = 33 / 192
/ 256 on the fp32 scan, M = 16 / 32, ragged query blocks, id offsets).  The test hook MIVQ_ADC_NO_RERUN skips the re-run, which
shows the certificate really carries the ordinary cases and really refuses the adversarial
ones; MIVQ_ADC_SMALL_RERUN_GRID puts the re-run on one column of workgroups, so each walks
several list-slot blocks (the path large databases with many uncertified queries take)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _h(t):
    return t.detach().cpu().numpy()


EXACT, NO_RERUN, SMALL_GRID = 1, 2, 4  # MIVQ_ADC_FORCE_EXACT / _NO_RERUN / _SMALL_RERUN_GRID


def _search(lut_d, codes_d, k, id_offset=0, flags=0):
    from haag_vq import _native

    d, i = _native.adc_search(lut_d, codes_d, k, 8, id_offset=id_offset, flags=flags)
    torch.cuda.synchronize()
    return _h(d), _h(i).view(np.uint32)


def _check(dev, oracle, lut, u8, k, id_offset=0):
    d_ref, i_ref = oracle.adc_search(lut, u8, k, id_offset)
    lut_d, codes_d = _t(lut, dev), _t(u8, dev)
    d_f, i_f = _search(lut_d, codes_d, k, id_offset)
    d_e, i_e = _search(lut_d, codes_d, k, id_offset, EXACT)
    np.testing.assert_array_equal(d_f, d_ref)
    np.testing.assert_array_equal(i_f, i_ref)
    np.testing.assert_array_equal(d_e, d_ref)
    np.testing.assert_array_equal(i_e, i_ref)
    return lut_d, codes_d, d_ref, i_ref


def _lut(oracle, rng, nq, M, dsub, metric=1):
    C = rng.standard_normal((M, 256, dsub)).astype(np.float32)
    Q = rng.standard_normal((nq, M * dsub)).astype(np.float32)
    return oracle.adc_lut(Q, C, metric)


@pytest.mark.parametrize("M,k", [(16, 1), (16, 10), (16, 32), (16, 33), (16, 256), (32, 1), (32, 10), (32, 32), (32, 192)])
@pytest.mark.parametrize("metric", [1, 0])
def test_filtered_adc_shapes(dev, oracle, M, k, metric):
    rng = np.random.default_rng(M * 1000 + k)
    nq, n = 37, 20011
    lut = _lut(oracle, rng, nq, M, 8, metric)
    u8 = rng.integers(0, 256, size=(n, M)).astype(np.uint8)
    u8[n - 1] = u8[0]  # duplicate rows far apart: id tie-break
    u8[n // 2] = u8[0]
    lut_d, codes_d, d_ref, i_ref = _check(dev, oracle, lut, u8, k, id_offset=123457)
    if k <= 32:
        # ordinary data (k <= 32 takes the filtered path): every query certified by the filter alone
        d_n, i_n = _search(lut_d, codes_d, k, 123457, NO_RERUN)
        assert not np.isnan(d_n).any()  # every query certified
        np.testing.assert_array_equal(i_n, i_ref)
        np.testing.assert_array_equal(d_n, d_ref)


def test_filtered_adc_all_rows_identical(dev, oracle):
    """Every row the same code: every part's list is full of equal keys, no certificate can
    hold -- all queries go to the fp32 re-run, and the answer is rows 0..k-1."""
    rng = np.random.default_rng(1)
    nq, n, M, k = 21, 30000, 16, 10
    lut = _lut(oracle, rng, nq, M, 4)
    u8 = np.tile(rng.integers(0, 256, size=(1, M)).astype(np.uint8), (n, 1))
    lut_d, codes_d, d_ref, i_ref = _check(dev, oracle, lut, u8, k)
    assert (i_ref == np.arange(k, dtype=np.uint32)).all()
    d_n, i_n = _search(lut_d, codes_d, k, 0, NO_RERUN)
    assert np.isnan(d_n).all()  # the filter alone vouches for none of them (unset rows are NaN)
    # the re-run on one workgroup column: each workgroup walks all three 8-query slot blocks
    d_s, i_s = _search(lut_d, codes_d, k, 0, SMALL_GRID)
    np.testing.assert_array_equal(d_s, d_ref)
    np.testing.assert_array_equal(i_s, i_ref)


def test_filtered_adc_few_distinct_rows_and_near_ties(dev, oracle):
    """A handful of distinct code rows (massive ties) and LUT entries that differ by a few ulps
    (every row inside the quantisation window)."""
    rng = np.random.default_rng(2)
    nq, n, M, k = 19, 25000, 16, 17
    lut = _lut(oracle, rng, nq, M, 4)
    base = rng.integers(0, 256, size=(5, M)).astype(np.uint8)
    u8 = base[rng.integers(0, 5, size=n)]
    _check(dev, oracle, lut, u8, k)
    near = np.full((nq, M, 256), 0.5, np.float32)
    near += rng.integers(0, 4, size=near.shape).astype(np.float32) * np.float32(2 ** -24)
    near[3] *= np.float32(1e30)  # one query with huge entries
    near[4] *= np.float32(1e-30)  # and one with tiny ones
    u8 = rng.integers(0, 256, size=(n, M)).astype(np.uint8)
    _check(dev, oracle, near, u8, k)


def test_filtered_adc_nonfinite_luts(dev, oracle):
    """+inf / NaN entries: those queries take the fp32 scan (NaN distances rank as +inf)."""
    rng = np.random.default_rng(3)
    nq, n, M, k = 18, 6000, 16, 10
    lut = _lut(oracle, rng, nq, M, 4)
    lut[2, 5, :] = np.inf
    lut[7, 0, 17] = np.nan
    lut[9, 3, 200] = -np.inf
    u8 = rng.integers(0, 256, size=(n, M)).astype(np.uint8)
    _check(dev, oracle, lut, u8, k)


@pytest.mark.parametrize("n", [1, 9, 1023, 4097])
def test_filtered_adc_small_databases(dev, oracle, n):
    rng = np.random.default_rng(n)
    nq, M, k = 33, 16, 10
    lut = _lut(oracle, rng, nq, M, 4)
    u8 = rng.integers(0, 256, size=(n, M)).astype(np.uint8)
    _check(dev, oracle, lut, u8, k, id_offset=7)


def test_filtered_adc_rerun_many_slot_blocks_large_db(dev):
    """Many uncertified queries over a database large enough for several re-run chunks, with
    the re-run grid forced to one column (each workgroup walks ~10 slot blocks): equal to the
    fp32 scan of every query, and to a torch restatement of the canonical sums (m in order,
    stable sort: ties to the smaller id)."""
    from haag_vq import _native

    g = torch.Generator(device=dev).manual_seed(5)
    n, M, k, nq = 300_000, 16, 10, 80
    base = torch.randint(0, 256, (64, M), device=dev, dtype=torch.uint8, generator=g)
    # 64 distinct rows repeated: massive ties, so most queries cannot be certified and go to the
    # re-run (a query whose best row's copies fill its whole top-k with a clear gap can be)
    codes = base[torch.randint(0, 64, (n,), device=dev, generator=g)].contiguous()
    lut = torch.rand((nq, M, 256), device=dev, generator=g, dtype=torch.float32)
    d_f, i_f = _search(lut, codes, k, 11, SMALL_GRID)
    d_e, i_e = _search(lut, codes, k, 11, EXACT)
    d_n, _ = _search(lut, codes, k, 11, NO_RERUN)
    failed = np.isnan(d_n).all(axis=1)
    assert failed.sum() >= nq // 2, failed.sum()  # >= 5 slot blocks walked by one workgroup column
    np.testing.assert_array_equal(d_f, d_e)
    np.testing.assert_array_equal(i_f, i_e)
    ci = codes.long()
    for q in (0, 37, 79):
        dist = lut[q, 0][ci[:, 0]].clone()
        for m in range(1, M):
            dist += lut[q, m][ci[:, m]]
        order = torch.sort(dist, stable=True).indices[:k]
        np.testing.assert_array_equal(i_f[q], _h(order).astype(np.uint32) + 11)
        np.testing.assert_array_equal(d_f[q], _h(dist[order]))



@pytest.mark.parametrize("nq,n,M", [(4200, 30_000, 16), (2000, 200_000, 16), (4200, 30_000, 32)])
def test_filtered_adc_grid_shapes(dev, nq, n, M):
    """Grids of more than one round of CUs: 4200 queries (263 query blocks x 1 chunk) take the
    pinned-prefetch scan kernel (M = 16 and M = 32); 2000 queries over 200k rows take the
    one-round chunk rule (2 -> 4 chunks, then two rounds, pinned).  Equal to the fp32 scan for every query and to a
    torch restatement of the canonical sums for a few."""
    g = torch.Generator(device=dev).manual_seed(nq + M)
    k = 10
    codes = torch.randint(0, 256, (n, M), device=dev, dtype=torch.uint8, generator=g)
    codes[n - 1] = codes[3]  # a duplicate row: tie to the smaller id
    lut = torch.rand((nq, M, 256), device=dev, generator=g, dtype=torch.float32)
    d_f, i_f = _search(lut, codes, k, 5)
    d_e, i_e = _search(lut, codes, k, 5, EXACT)
    np.testing.assert_array_equal(d_f, d_e)
    np.testing.assert_array_equal(i_f, i_e)
    ci = codes.long()
    for q in (0, nq // 2, nq - 1):
        dist = lut[q, 0][ci[:, 0]].clone()
        for m in range(1, M):
            dist += lut[q, m][ci[:, m]]
        order = torch.sort(dist, stable=True).indices[:k]
        np.testing.assert_array_equal(i_f[q], _h(order).astype(np.uint32) + 5)
        np.testing.assert_array_equal(d_f[q], _h(dist[order]))
