"""`vq-benchmark ivf-bench` on the GPU: every runner of the build on a small Gaussian set
(reference /root/reference/src/haag_vq/benchmarks/ivf_benchmark.py:95-310).  The ground truth
written to the dataset directory equals a float64 numpy brute force; the pq_flat row's MSE and
recall equal an independent decode of the same (deterministic) quantizer followed by a float64
exact search; compression ratios and the IVF-PQ memory estimate follow the reference's formulas."""
import csv

import numpy as np
import pytest

from haag_vq.benchmarks import ivf_benchmark as ib


def _knn(X, Q, k):
    d = ((Q[:, None, :].astype(np.float64) - X[None, :, :].astype(np.float64)) ** 2).sum(-1)
    return np.argsort(d, axis=1, kind="stable")[:, :k]


@pytest.mark.gpu
def test_ivf_bench_runners(dev, tmp_path):
    rng = np.random.default_rng(11)
    N, D, nq, k = 6000, 64, 50, 10
    X = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((nq, D)).astype(np.float32)
    np.save(tmp_path / "train.npy", X)
    np.save(tmp_path / "queries.npy", Q)
    out = ib.ivf_benchmark(dataset=str(tmp_path), methods="pq_flat,opq_flat,sq_flat,faiss_ivfpq,rabitq,saq", bpd=4,
                           k=k, nlist=32, nprobe=8, output=str(tmp_path / "res.csv"), num_queries=nq, gt_k=20)
    gt = np.load(tmp_path / "ground_truth.npy")
    assert gt.shape == (nq, 20) and np.array_equal(gt, _knn(X, Q, 20))
    rows = {r["method"]: r for r in csv.DictReader(open(out))}
    assert list(rows) == ["pq_flat", "opq_flat", "sq_flat", "faiss_ivfpq", "rabitq"]
    for r in rows.values():
        assert 0.0 <= float(r["recall_at_k"]) <= 1.0 and float(r["qps"]) > 0
        assert (int(r["k"]), int(r["N"]), int(r["D"])) == (k, N, D)
    M = ib._bpd_to_pq_M(D, 4)
    assert M == 32
    for m in ("pq_flat", "opq_flat", "sq_flat"):  # 32 code bytes per 256-B row
        assert int(rows[m]["memory_bytes"]) == N * 32 and float(rows[m]["compression_ratio"]) == 8.0
    assert int(rows["faiss_ivfpq"]["memory_bytes"]) == N * M + 32 * D * 4 and rows["faiss_ivfpq"]["mse"] == ""
    assert float(rows["sq_flat"]["recall_at_k"]) > 0.5 and float(rows["pq_flat"]["recall_at_k"]) > 0.3

    from haag_vq.methods.product_quantization import ProductQuantizer

    pq = ProductQuantizer(M=M, B=8)
    pq.fit(X)
    R = pq.decompress(pq.compress(X)).astype(np.float64)
    mse = float(((X.astype(np.float64) - R) ** 2).sum(1).mean())
    assert float(rows["pq_flat"]["mse"]) == pytest.approx(mse, rel=1e-9)
    rec = ib._recall_at_k(gt, _knn(R, Q, k), k)
    assert float(rows["pq_flat"]["recall_at_k"]) == pytest.approx(rec, abs=0.01)  # near-ties aside
