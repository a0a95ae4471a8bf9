"""Search-index benchmark driver, host logic (no GPU): method construction rules, dataset
formats, argument checks (reference: /root/reference/src/haag_vq/benchmarks/run_benchmarks.py
:43-90 load_dataset, :118-246 build_method_configs, :317-330 sweep-mode check)."""
import numpy as np
import pytest

from haag_vq.benchmarks import run_benchmarks as rb


def test_build_method_configs_rules(capsys):
    from haag_vq.methods.search import FaissIvfPqIndex, FlatQuantizedIndex, RaBitQIndex

    cfg = rb.build_method_configs(["pq_flat", "opq_flat", "sq_flat", "faiss_ivfpq", "rabitq", "pq_ivf", "saq",
                                   "rabitq_ivf", "bogus"], D=100, bpd=3.0, K=64, nprobe=7)
    assert list(cfg) == ["pq_flat", "opq_flat", "sq_flat", "faiss_ivfpq", "rabitq"]
    assert isinstance(cfg["pq_flat"], FlatQuantizedIndex) and cfg["pq_flat"].quantizer.M == 37  # 300 // 8
    assert cfg["opq_flat"].quantizer.M == 25  # 37 lowered until it divides 100
    assert cfg["sq_flat"].quantizer.num_bits == 4
    assert isinstance(cfg["faiss_ivfpq"], FaissIvfPqIndex) and cfg["faiss_ivfpq"].nprobe == 7
    assert isinstance(cfg["rabitq"], RaBitQIndex)
    err = capsys.readouterr().err
    assert "pq_ivf unavailable" in err and "saq unavailable" in err and "unknown method 'bogus'" in err
    assert rb._pq_M(64, 16.0) == 64 and rb._pq_M(4, 0.5) == 1  # clamped to [1, D]
    assert [rb._sq_bits(b) for b in (2, 4.5, 5, 12, 12.5)] == [4, 4, 8, 8, 16]


def test_load_dataset_formats(tmp_path):
    from haag_vq.utils.faiss_export import write_fvecs, write_ivecs

    X, Q, g = rb.load_dataset("synthetic")
    assert X.shape == (2000, 64) and Q.shape == (100, 64) and g is None and X.dtype == np.float32
    rng = np.random.default_rng(1)
    A, B = rng.standard_normal((30, 8)), rng.standard_normal((5, 8))
    d1 = tmp_path / "npy"
    d1.mkdir()
    np.save(d1 / "train.npy", A)
    np.save(d1 / "queries.npy", B)
    np.save(d1 / "groundtruth.npy", np.arange(10, dtype=np.int32).reshape(5, 2))
    X, Q, g = rb.load_dataset(str(d1))
    assert np.array_equal(X, A.astype(np.float32)) and Q.shape == (5, 8) and g.dtype == np.int64
    d2 = tmp_path / "fvecs"
    d2.mkdir()
    write_fvecs(d2 / "base.fvecs", A.astype(np.float32))
    write_fvecs(d2 / "query.fvecs", B.astype(np.float32))
    write_ivecs(d2 / "groundtruth.ivecs", np.arange(10, dtype=np.int32).reshape(5, 2))
    X, Q, g = rb.load_dataset(str(d2))
    assert np.array_equal(X, A.astype(np.float32)) and np.array_equal(g, np.arange(10).reshape(5, 2))
    with pytest.raises(ValueError):
        rb.load_dataset(str(tmp_path))
    with pytest.raises(FileNotFoundError):
        rb.load_dataset(str(tmp_path / "missing"))


def test_sweep_needs_one_method(tmp_path):
    np.save(tmp_path / "train.npy", np.zeros((10, 4), np.float32))
    np.save(tmp_path / "queries.npy", np.zeros((2, 4), np.float32))
    np.save(tmp_path / "groundtruth.npy", np.zeros((2, 10), np.int64))  # no GPU call for the GT
    with pytest.raises(SystemExit):
        rb.main(["--dataset", str(tmp_path), "--methods", "pq_flat,sq_flat", "--sweep-bpd", "2,4"])
