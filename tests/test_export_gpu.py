"""The reference's own tests of the QPS proxy and the codebook export, run against the MI355X
build (reference tests/test_faiss_export.py and
tests/test_performance_metrics.py).  `test_export_codebook_uses_ivf` is not mirrored: it
asserts a faiss ``IndexIVF`` object, and faiss is absent from this build by design."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_query_codebook_with_model(tmp_path):  # test_faiss_export.py:9-34
    from haag_vq.methods.scalar_quantization import ScalarQuantizer
    from haag_vq.utils.faiss_export import export_codebook, query_codebook

    data = np.array([[0.0, 0.0, 0.0], [1.0, 1.0, 1.0], [0.5, 0.5, 0.5]], dtype=np.float32)
    q = ScalarQuantizer()
    q.fit(data)
    cb = export_codebook(q, tmp_path)["codebook_vectors"]
    d, i = query_codebook(np.array([[0.9, 0.9, 0.9]], dtype=np.float32), model=q, codebook_vectors=cb, topk=1)
    assert d.shape == (1, 1) and i.shape == (1, 1)
    assert i[0, 0] == 1  # the max vector is closest to the query


def test_query_codebook_from_disk(tmp_path):  # test_faiss_export.py:37-63
    from haag_vq.methods.scalar_quantization import ScalarQuantizer
    from haag_vq.utils.faiss_export import export_codebook, query_codebook

    data = np.array([[0.0, 0.0], [2.0, 2.0]], dtype=np.float32)
    q = ScalarQuantizer()
    q.fit(data)
    path = export_codebook(q, tmp_path, codebook_filename="cb.fvecs")["codebook"]
    d, i = query_codebook(np.array([[0.1, 0.1], [1.9, 1.9]], dtype=np.float32), codebook_path=path, topk=2)
    assert d.shape == (2, 2) and i.shape == (2, 2)
    assert i[0, 0] == 0 and i[1, 0] == 1


@pytest.mark.parametrize("topk", [1, 2])
def test_query_codebook_product_quantizer(tmp_path, topk):  # test_faiss_export.py:86-110
    from haag_vq.methods.product_quantization import ProductQuantizer
    from haag_vq.utils.faiss_export import export_codebook, query_codebook

    rng = np.random.default_rng(0)
    data = rng.standard_normal((32, 8), dtype=np.float32)
    q = ProductQuantizer(M=2, B=2)  # ksub = 4
    q.fit(data)
    cb = export_codebook(q, tmp_path)["codebook_vectors"]
    queries = data[:5]
    d, i = query_codebook(queries, model=q, codebook_vectors=cb, topk=topk)
    assert d.shape == (5, q.M * topk) and i.shape == (5, q.M * topk)
    ksub = 2 ** q.B
    assert np.all(i[:, :topk] < ksub)
    assert np.all((i[:, topk:] >= ksub) & (i[:, topk:] < 2 * ksub))
    # and the values: per subspace, the nearest centroids of the query's sub-vector
    C = cb.reshape(q.M, ksub, -1)
    for m in range(q.M):
        dm = ((queries[:, None, m * 4:(m + 1) * 4] - C[m][None]) ** 2).sum(-1)
        ref = np.argsort(dm, axis=1, kind="stable")[:, :topk] + m * ksub
        np.testing.assert_array_equal(i[:, m * topk:(m + 1) * topk], ref)
        np.testing.assert_allclose(d[:, m * topk:(m + 1) * topk], np.sort(dm, axis=1)[:, :topk], rtol=1e-5, atol=1e-6)


def test_query_codebook_opq_offsets(tmp_path):
    from haag_vq.methods.optimized_product_quantization import OptimizedProductQuantizer
    from haag_vq.utils.faiss_export import export_codebook, query_codebook

    rng = np.random.default_rng(1)
    data = rng.standard_normal((600, 16), dtype=np.float32)
    q = OptimizedProductQuantizer(M=4, B=8)
    q.niter = 2
    q.fit(data)
    cb = export_codebook(q, tmp_path)["codebook_vectors"]
    assert cb.shape == (4 * 256, 4)
    _, i = query_codebook(data[:7], model=q, codebook_vectors=cb, topk=1)
    assert i.shape == (7, 4)
    for m in range(4):
        assert np.all((i[:, m] >= m * 256) & (i[:, m] < (m + 1) * 256))
    # top-1 per subspace = the PQ code of the rotated query
    np.testing.assert_array_equal(i - np.arange(4) * 256, q.compress(data[:7]).astype(np.int64))


def test_compression_and_decompression_latency():  # test_performance_metrics.py:8-29
    from haag_vq.methods.scalar_quantization import ScalarQuantizer
    from haag_vq.metrics.performance import time_compress, time_decompress

    X = np.array([[0.0, 0.2, 0.4], [0.5, 0.6, 0.7], [1.0, 0.8, 0.6]], dtype=np.float32)
    q = ScalarQuantizer()
    q.fit(X)
    codes, tc = time_compress(q, X)
    assert codes.shape == X.shape and tc >= 0.0
    rec, td = time_decompress(q, codes)
    assert rec.shape == X.shape and td >= 0.0


def test_measure_qps(tmp_path):  # test_performance_metrics.py:32-57
    from haag_vq.methods.scalar_quantization import ScalarQuantizer
    from haag_vq.metrics.performance import measure_qps
    from haag_vq.utils.faiss_export import export_codebook

    X = np.array([[0.0, 0.0], [1.0, 1.0], [2.0, 2.0]], dtype=np.float32)
    q = ScalarQuantizer()
    q.fit(X)
    cb = export_codebook(q, tmp_path)["codebook_vectors"]
    m = measure_qps(np.array([[0.1, 0.2], [1.9, 2.1]], dtype=np.float32), model=q, codebook_vectors=cb, repeats=2)
    assert m["qps"] > 0 and m["avg_query_latency_ms"] >= 0


def test_measure_qps_rabitq_compresses_queries():  # performance.py:60-63: RaBitQ times compress(queries)
    from haag_vq.methods.rabit_quantization import RaBitQuantizer
    from haag_vq.metrics.performance import measure_qps

    X = np.random.default_rng(2).standard_normal((50, 64)).astype(np.float32)
    q = RaBitQuantizer()
    q.fit(X)
    m = measure_qps(X[:10], model=q, repeats=2)
    assert m["qps"] > 0 and set(m) == {"qps", "qps_std", "avg_query_latency_ms", "latency_ms_std"}


def test_export_codebook_pq_roundtrip(tmp_path):
    from haag_vq.methods.product_quantization import ProductQuantizer
    from haag_vq.utils.faiss_export import export_codebook, load_fvecs, load_ivecs

    X = np.random.default_rng(3).standard_normal((500, 32)).astype(np.float32)
    q = ProductQuantizer(M=4, B=8)
    q.fit(X)
    codes = q.compress(X)
    res = export_codebook(q, tmp_path, codes=codes)
    cb = load_fvecs(res["codebook"])
    np.testing.assert_array_equal(cb, np.concatenate([np.asarray(c, np.float32) for c in q.codebooks]))
    np.testing.assert_array_equal(load_ivecs(res["codes"]), codes.astype(np.int32))
