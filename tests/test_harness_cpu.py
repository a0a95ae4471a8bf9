"""Host-side harness logic on CPU (no GPU): the sweep's config grids, the registry's module
paths, the CLI surface, the on-disk formats (fvecs / ivecs, codebook export) and the
streaming reader.  Mirrors the reference's structural tests where they exist
(tests/test_method_registry.py, tests/test_faiss_export.py round trips)."""

import numpy as np
import pytest


def test_pq_opq_grids():
    from haag_vq.benchmarks.sweep import _generate_opq_configs, _generate_pq_configs

    g = _generate_pq_configs("8,16", "6,8")
    assert [(c["subquantizers"], c["bits"]) for c in g] == [(8, 6), (8, 8), (16, 6), (16, 8)]
    assert g[0]["name"] == "PQ(subquantizers=8, bits=6)"
    o = _generate_opq_configs("32", "8")
    assert o == [{"name": "OPQ(subquantizers=32, bits=8)", "subquantizers": 32, "bits": 8}]


def test_sq_grid_is_8bit_only(capsys):
    from haag_vq.benchmarks.sweep import _generate_sq_configs

    assert _generate_sq_configs("4,8,16") == [{"name": "SQ(8-bit)", "num_bits": 8}]
    assert "Skipping 4-bit" in capsys.readouterr().out
    assert _generate_sq_configs("4") == [{"name": "SQ(8-bit)", "num_bits": 8}]  # the fallback


def test_rabitq_grid_parses_names_and_numbers():
    from haag_vq.benchmarks.sweep import _generate_rabitq_configs
    from haag_vq.utils.faiss_utils import MetricType

    g = _generate_rabitq_configs("L2, 0 ,inner_product")
    assert [c["metric_type"] for c in g] == [MetricType.L2, MetricType.INNER_PRODUCT, MetricType.INNER_PRODUCT]
    assert g[0]["name"] == "RabitQ(metric=L2)"
    with pytest.raises(ValueError, match="Unknown RabitQ metric type"):
        _generate_rabitq_configs("cosine")


def test_sweep_rejects_unknown_method_and_saq(tmp_path):
    from typer.testing import CliRunner

    from haag_vq.cli import app

    r = CliRunner().invoke(app, ["sweep", "--dataset", "nope", "--codebooks-dir", str(tmp_path)])
    assert r.exit_code != 0 and isinstance(r.exception, ValueError)
    r = CliRunner().invoke(app, ["sweep", "--dataset", "dbpedia-100k", "--method", "pq",
                                 "--cache-dir", str(tmp_path), "--codebooks-dir", str(tmp_path)])
    assert isinstance(r.exception, FileNotFoundError)  # no network: a local file is required


def test_cli_commands():
    from typer.testing import CliRunner

    from haag_vq.cli import app

    out = CliRunner().invoke(app, ["--help"]).output
    assert "sweep" in out and "streaming-sweep" in out
    out = CliRunner().invoke(app, ["sweep", "--help"]).output
    for opt in ("--method", "--dataset", "--pq-subquantizers", "--pq-bits", "--sq-bits", "--rabitq-metric-type",
                "--opq-quantizers", "--with-recall", "--num-pairs", "--rank-k", "--ground-truth-path", "--db-path"):
        assert opt in out, opt


def test_method_registry_saq_module_path():
    from haag_vq.benchmarks import method_registry_saq as mrs

    assert "rabitq" in mrs.SAQ_METHODS
    with pytest.raises(ValueError):
        mrs.build_saq_quantizer("saq_paper", 4, 64)
    with pytest.raises(ValueError):
        mrs.build_saq_quantizer("nope", 4, 64)


def test_largest_divisor_leq_known_answers():  # reference tests/test_method_registry.py:11-15
    from haag_vq.benchmarks.method_registry import _pq_subquantizers, largest_divisor_leq

    assert largest_divisor_leq(1536, 600) == 512
    assert largest_divisor_leq(1536, 192) == 192
    assert largest_divisor_leq(100, 7) == 5
    assert largest_divisor_leq(7, 100) == 7
    assert _pq_subquantizers(1.0, 1536) == 192


def test_fvecs_ivecs_roundtrip(tmp_path):
    from haag_vq.utils.faiss_export import load_fvecs, load_ivecs, write_fvecs, write_ivecs

    X = np.random.default_rng(0).standard_normal((17, 5)).astype(np.float32)
    I = np.random.default_rng(1).integers(-5, 1 << 20, size=(9, 3)).astype(np.int32)
    np.testing.assert_array_equal(load_fvecs(write_fvecs(tmp_path / "a.fvecs", X)), X)
    np.testing.assert_array_equal(load_ivecs(write_ivecs(tmp_path / "a.ivecs", I)), I)
    raw = (tmp_path / "a.fvecs").read_bytes()
    assert len(raw) == 17 * 6 * 4 and np.frombuffer(raw[:4], np.int32)[0] == 5  # faiss .fvecs layout
    (tmp_path / "bad.fvecs").write_bytes(raw[:-4])
    with pytest.raises(ValueError):
        load_fvecs(tmp_path / "bad.fvecs")
    with pytest.raises(FileNotFoundError):
        load_fvecs(tmp_path / "missing.fvecs")


def test_export_codebook_of_duck_typed_pq(tmp_path):
    from haag_vq.utils.faiss_export import export_codebook, load_fvecs, load_ivecs

    class PQLike:  # what export_codebook reads of a ProductQuantizer: .codebooks
        codebooks = [np.full((4, 2), m, np.float32) for m in range(3)]

    codes = np.array([[0, 1, 2], [3, 3, 3]])
    res = export_codebook(PQLike(), tmp_path, codes=codes)
    np.testing.assert_array_equal(load_fvecs(res["codebook"]), np.concatenate(PQLike.codebooks))
    np.testing.assert_array_equal(load_ivecs(res["codes"]), codes.astype(np.int32))


def test_streaming_reader_npy_and_fvecs(tmp_path):
    from haag_vq.benchmarks.streaming_sweep import open_vector_stream
    from haag_vq.utils.faiss_export import write_fvecs

    X = np.random.default_rng(2).standard_normal((31, 7)).astype(np.float32)
    np.save(tmp_path / "x.npy", X)
    write_fvecs(tmp_path / "x.fvecs", X)
    for name in ("x.npy", "x.fvecs"):
        s = open_vector_stream(tmp_path / name)
        assert s.shape == (31, 7)
        np.testing.assert_array_equal(np.asarray(s[10:20]), X[10:20])


def test_dataset_default_metric_is_reference_euclidean():
    from sklearn.metrics import pairwise_distances

    from haag_vq.data.datasets import Dataset, is_euclidean

    d = Dataset(np.zeros((3, 2)), ground_truth=np.zeros((3, 1), np.int64), num_queries=3)
    assert d.distance_metric is pairwise_distances and is_euclidean(d.distance_metric)
    assert not is_euclidean(lambda a, b: pairwise_distances(a, b, metric="cosine"))
