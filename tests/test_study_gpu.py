"""The study driver and the search-index harness (the reference's tests/test_quantizer_study.py,
tests/test_study_config.py and tests/test_results_timestamping.py), on the MI355X path: the
quantizers encode / decode through libmivq and the rankings come from mivq_flat_search."""

import re
import textwrap

import numpy as np
import pytest

ISO_UTC = re.compile(r"^\d{4}-\d{2}-\d{2}T\d{2}:\d{2}:\d{2}Z$")


def _unit_rows(n, d, seed):
    X = np.random.default_rng(seed).standard_normal((n, d)).astype(np.float32)
    return X / (np.linalg.norm(X, axis=1, keepdims=True) + 1e-12)


def _write_fvecs(path, X):
    d = X.shape[1]
    rec = np.empty((X.shape[0], d + 1), dtype=np.float32)
    rec[:, 0] = np.array([d], dtype=np.int32).view(np.float32)[0]
    rec[:, 1:] = X
    rec.tofile(path)


def test_load_study_config(tmp_path):
    from haag_vq.benchmarks.study_config import StudyConfig, load_study_config

    p = tmp_path / "cfg.yaml"
    p.write_text(textwrap.dedent("""
        dataset:
          name: toy
          base_fvecs: /tmp/base.fvecs
          query_fvecs: /tmp/query.fvecs
          n_queries: 1000
        methods: [pq, sq]
        bpd: [1, 2, 4, 8]
    """))
    cfg = load_study_config(p)
    assert isinstance(cfg, StudyConfig)
    assert cfg.methods == ["pq", "sq"] and cfg.bpd == [1, 2, 4, 8]
    assert cfg.ks == [1, 10, 100] and cfg.chunk_size == 50_000 and cfg.mse_sample == 100_000
    assert cfg.output_dir == "results" and cfg.dataset["n_queries"] == 1000


@pytest.mark.gpu
def test_run_study_arrays_pq_sq():
    from haag_vq.benchmarks.quantizer_study import run_study_arrays

    rng = np.random.default_rng(0)
    X = rng.standard_normal((1000, 48)).astype(np.float32)
    Q = rng.standard_normal((50, 48)).astype(np.float32)
    df = run_study_arrays(X, Q, methods=["pq", "sq"], bpd_values=[4, 8], ks=(1, 10), chunk_size=256,
                          mse_sample=1000)
    assert len(df) == 4
    for col in ("method", "bpd", "compression_factor", "code_bytes", "mse", "recall_at_1", "recall_at_10",
                "n_db", "n_queries", "D", "timestamp"):
        assert col in df.columns
    assert df["recall_at_10"].between(0, 1).all()
    assert (df["compression_factor"] > 1).all() and df["mse"].min() >= 0
    # more bits per dimension: no worse reconstruction, no better compression
    for m in ("pq", "sq"):
        sub = df[df["method"] == m].sort_values("bpd")
        assert sub["mse"].iloc[1] <= sub["mse"].iloc[0] + 1e-9
        assert sub["compression_factor"].iloc[1] <= sub["compression_factor"].iloc[0]


@pytest.mark.gpu
def test_run_study_from_config_and_cli(tmp_path):
    from haag_vq.benchmarks import quantizer_study as qs

    X, Q = _unit_rows(600, 32, 1), _unit_rows(20, 32, 2)
    _write_fvecs(tmp_path / "base.fvecs", X)
    _write_fvecs(tmp_path / "query.fvecs", Q)
    np.testing.assert_array_equal(qs._load_fvecs(str(tmp_path / "base.fvecs")), X)
    cfg = tmp_path / "study.yaml"
    cfg.write_text(textwrap.dedent(f"""
        dataset:
          name: toy
          base_fvecs: {tmp_path / 'base.fvecs'}
          query_fvecs: {tmp_path / 'query.fvecs'}
          n_queries: 10
        methods: [sq]
        bpd: [8]
        ks: [1, 10]
        chunk_size: 128
        output_dir: {tmp_path / 'out'}
    """))
    df = qs.run_study(qs.load_study_config(cfg))
    assert list(df["dataset"]) == ["toy"] and int(df["n_queries"].iloc[0]) == 10
    assert df["recall_at_10"].iloc[0] > 0.9  # 8-bit SQ keeps the exact neighbours
    qs.main(["--config", str(cfg)])
    assert len(list((tmp_path / "out").glob("results_*.csv"))) == 1


@pytest.mark.gpu
def test_ground_truth_matches_numpy():
    from haag_vq.benchmarks.search_bench import compute_ground_truth

    X, Q = _unit_rows(500, 24, 3), _unit_rows(7, 24, 4)
    d2 = ((Q[:, None, :].astype(np.float64) - X[None].astype(np.float64)) ** 2).sum(-1)
    np.testing.assert_array_equal(compute_ground_truth(X, Q, k=5)[:, 0], d2.argmin(1))
    ip = Q.astype(np.float64) @ X.T.astype(np.float64)
    np.testing.assert_array_equal(compute_ground_truth(X, Q, k=5, metric="ip")[:, 0], ip.argmax(1))
    assert compute_ground_truth(X[:3], Q, k=10).shape == (7, 3)


@pytest.mark.gpu
def test_benchmark_index_compare_and_sweep_timestamps():
    from haag_vq.benchmarks.search_bench import benchmark_index, compare_methods, compute_ground_truth, sweep_bpd
    from haag_vq.methods.scalar_quantization import ScalarQuantizer
    from haag_vq.methods.search import FlatQuantizedIndex

    X, Q = _unit_rows(64, 8, 0), _unit_rows(4, 8, 1)
    gt = compute_ground_truth(X, Q, k=3)
    r = benchmark_index(FlatQuantizedIndex(ScalarQuantizer(num_bits=8)), X, Q, gt, k=3)
    assert r["method"] == "FlatQuantizedIndex" and 0.0 <= r["recall_at_k"] <= 1.0 and r["qps"] > 0
    assert r["compression_ratio"] > 1 and r["mse"] >= 0 and (r["k"], r["N"], r["D"]) == (3, 64, 8)
    df = compare_methods({"sq_flat": FlatQuantizedIndex(ScalarQuantizer(num_bits=8))}, X, Q, gt, k=3)
    assert list(df["method"]) == ["sq_flat"] and all(ISO_UTC.match(t) for t in df["timestamp"])
    df2 = sweep_bpd(lambda _b: FlatQuantizedIndex(ScalarQuantizer(num_bits=8)), [4.0, 8.0], X, Q, gt, k=3)
    assert list(df2["bpd"]) == [4.0, 8.0] and df2["timestamp"].nunique() == 1


@pytest.mark.gpu
def test_precompute_gt_cli_matches_numpy(tmp_path):
    """`vq-benchmark precompute-gt` on a memory-mapped .npy: database streamed in slices (a short
    last slice included) and merged on the device, equal to a numpy fp64 brute force."""
    from typer.testing import CliRunner

    from haag_vq.benchmarks import precompute_ground_truth as pg
    from haag_vq.cli import app

    X = _unit_rows(3000, 40, 9)
    np.save(tmp_path / "v.npy", X)
    ids, dists = pg.exact_knn_l2(X, X[:25], k=7, batch_size=10, slice_rows=1024)
    d2 = ((X[:25, None, :].astype(np.float64) - X[None].astype(np.float64)) ** 2).sum(-1)
    ref = np.argsort(d2, axis=1, kind="stable")[:, :7]
    assert (ids[:, 0] == ref[:, 0]).all()
    np.testing.assert_allclose(dists, np.take_along_axis(d2, ids, 1), rtol=1e-5, atol=1e-5)
    assert (np.diff(dists, axis=1) >= 0).all()
    r = CliRunner().invoke(app, ["precompute-gt", "--vectors-path", str(tmp_path / "v.npy"), "--output-path",
                                 str(tmp_path / "gt" / "g.npy"), "--num-queries", "25", "--k", "7"])
    assert r.exit_code == 0, r.output
    np.testing.assert_array_equal(np.load(tmp_path / "gt" / "g.npy"), ids)
    assert np.load(tmp_path / "gt" / "g.distances.npy").shape == (25, 7)


@pytest.mark.gpu
def test_precompute_gt_pads_k_beyond_database():
    """k > rows keeps the requested width like faiss IndexFlatL2.search: the real
    neighbours first, then id -1 with distance FLT_MAX."""
    from haag_vq.benchmarks import precompute_ground_truth as pg

    X = _unit_rows(6, 16, 3)
    ids, dists = pg.exact_knn_l2(X, X[:4], k=10, batch_size=3, slice_rows=4)
    assert ids.shape == (4, 10) and dists.shape == (4, 10)
    assert (ids[:, 6:] == -1).all() and (dists[:, 6:] == np.finfo(np.float32).max).all()
    assert (np.sort(ids[:, :6], axis=1) == np.arange(6)).all()
    assert (ids[:, 0] == np.arange(4)).all()
