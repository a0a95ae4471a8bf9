"""Pinning the hot path as far as the environment allows (faiss is absent):

* PQ codes on k-means-trained codebooks at the BASELINE shapes (PQ16 / PQ32 / PQ8 at
  D = 1536, >= 20k rows): bit-exact against the canonical oracle, and equal to an fp64
  brute-force nearest centroid on every (row, subspace) whose fp64 top-2 gap clears the
  rigorous fp32 rounding bound (an independent definition: any correct fp32 encoder,
  faiss' included, must agree there);
* ADC distances against fp64 decode + exact distances, within 1e-5 relative, at M = 16
  and 32, and the ADC top-k set equal to the decode-then-exact top-k up to near-ties;
* Extended RaBitQ: every index that differs from the reference's fixture sits at a level
  midpoint, i.e. within fp64 rounding of a searchsorted boundary.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

# relative bound on a canonical fp32 score difference, 2 (2 gamma_96 + u) ~ 2.3e-5 of
# |x|^2 + max|c|^2 for dsub <= 192 (oracle.pq_encode_fp64's gap unit), rounded up
CLEAR_GAP = 3e-5


def _unit_gauss(n, d, seed):
    X = np.random.default_rng(seed).standard_normal((n, d)).astype(np.float32)
    return X / np.linalg.norm(X, axis=1, keepdims=True)


@pytest.fixture(scope="module")
def data1536():
    return _unit_gauss(24576, 1536, 11)


@pytest.mark.parametrize("M", [16, 32, 8])
def test_pq_trained_codebooks_exact_and_fp64(dev, oracle, data1536, M):
    from haag_vq import _native
    from haag_vq.methods._kmeans import train_pq

    X = data1536
    Xd = torch.from_numpy(X).to(dev)
    C = train_pq(Xd[:16384], M, 8, niter=10, seed=1234, exact_assign=True).contiguous()
    codes = _native.pq_encode(Xd, C, _native.pq_prepare(C, 8), 8).cpu().numpy()
    Ch = C.cpu().numpy()
    np.testing.assert_array_equal(codes, oracle.pq_encode(X, Ch))
    c64, gap = oracle.pq_encode_fp64(X, Ch)
    clear = gap > CLEAR_GAP
    assert clear.mean() > 0.99, clear.mean()
    np.testing.assert_array_equal(codes[clear], c64[clear])


@pytest.mark.parametrize("M", [16, 32])
def test_adc_distances_match_fp64_decode(dev, oracle, data1536, M):
    from haag_vq import _native
    from haag_vq.methods._kmeans import train_pq

    X = data1536[:20000]
    Xd = torch.from_numpy(X).to(dev)
    C = train_pq(Xd[:16384], M, 8, niter=6, seed=1234, exact_assign=True).contiguous()
    codes = _native.pq_encode(Xd, C, _native.pq_prepare(C, 8), 8)
    Q = _unit_gauss(64, 1536, 99)
    k = 20
    lut = _native.adc_lut(torch.from_numpy(Q).to(dev), C, 8)
    dd, ii = _native.adc_search(lut, codes, k, 8)
    dd, ii = dd.cpu().numpy(), ii.cpu().numpy().view(np.uint32).astype(np.int64)
    Xhat = oracle.pq_decode(codes.cpu().numpy(), C.cpu().numpy()).astype(np.float64)
    Q64 = Q.astype(np.float64)
    d64 = ((Q64[:, None, :] - Xhat[ii]) ** 2).sum(-1)  # fp64 distance of every returned id
    np.testing.assert_allclose(dd, d64, rtol=1e-5)
    # the ADC ranking is the decode-then-exact ranking: the returned set is the exact top-k
    # except where the k-th and (k+1)-th fp64 distances are within the fp32 tolerance
    full = (Q64 ** 2).sum(1)[:, None] + (Xhat ** 2).sum(1)[None, :] - 2.0 * Q64 @ Xhat.T
    order = np.argsort(full, axis=1, kind="stable")
    for q in range(len(Q)):
        ref = set(order[q, :k].tolist())
        if ref != set(ii[q].tolist()):
            kth, nxt = full[q, order[q, k - 1]], full[q, order[q, k]]
            assert abs(nxt - kth) <= 2e-5 * abs(kth), (q, kth, nxt)


@pytest.mark.parametrize("nbits", [1, 2, 4, 8])
def test_extrabitq_mismatches_are_midpoint_ties(dev, golden_dir, nbits):
    from haag_vq import _native

    e = np.load(golden_dir / "extrabitq_golden.npz")
    X = e["X"].astype(np.float64)
    tag = f"b{nbits}"
    c, P, lv = (e[f"{tag}_{k}"] for k in ("c", "P", "levels"))
    codes = _native.extrabitq_encode(torch.from_numpy(e["X"]).to(dev), *(torch.from_numpy(a).to(dev) for a in (c, P, lv)),
                                     nbits).cpu().numpy()
    N, D = X.shape
    ib = (D * nbits + 7) // 8

    def unpack(cb):  # MSB-first B-bit indices (extended_rabitq.py:156-160)
        bits = np.unpackbits(cb[:, :ib], axis=1)[:, :D * nbits].reshape(N, D, nbits)
        return (bits.astype(np.int64) << np.arange(nbits - 1, -1, -1)).sum(-1)

    got, ref = unpack(codes), unpack(e[f"{tag}_codes"])
    bad = np.argwhere(got != ref)
    # s exactly as the reference computes it (extended_rabitq.py:133-141), in fp64
    r = X - c
    o = r / np.maximum(np.linalg.norm(r, axis=1), 1e-12)[:, None]
    s = (o @ P) * np.sqrt(D)
    mids = 0.5 * (lv[:-1] + lv[1:])
    for i, j in bad:
        dist = np.min(np.abs(mids - s[i, j]))
        assert dist <= 1e-12 * max(1.0, abs(s[i, j])), (i, j, s[i, j], dist)
        assert abs(int(got[i, j]) - int(ref[i, j])) == 1  # the two levels either side of it
    assert len(bad) <= 1e-3 * N * D
