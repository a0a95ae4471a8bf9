"""`vq-benchmark ivf-bench` host logic (no GPU): the bpd -> M rule, recall@k, the timestamped CSV
name, dataset loading with and without queries.npy, and that methods outside the build are
skipped (reference: /root/reference/src/haag_vq/benchmarks/ivf_benchmark.py:32-92, :367-451)."""
from datetime import datetime, timezone
from pathlib import Path

import numpy as np
from typer.testing import CliRunner

from haag_vq.benchmarks import ivf_benchmark as ib


def test_bpd_to_pq_M_rules():
    # M = D * bpd // 8, at least 1, lowered until it divides D
    assert ib._bpd_to_pq_M(128, 4) == 64
    assert ib._bpd_to_pq_M(100, 4) == 50
    assert ib._bpd_to_pq_M(96, 3) == 32  # 36, 35, 34, 33 do not divide 96
    assert ib._bpd_to_pq_M(7, 1) == 1
    assert ib._bpd_to_pq_M(1536, 1) == 192
    assert ib._bpd_to_pq_M(1536, 8) == 1536
    assert ib._bpd_to_pq_M(1024, 2) == 256


def test_recall_at_k():
    gt = np.array([[1, 2, 3], [4, 5, 6]])
    got = np.array([[3, 9, 1], [7, 8, 9]])
    assert ib._recall_at_k(gt, got, 3) == 2 / 6
    assert ib._recall_at_k(gt, got, 1) == 0.0
    assert ib._recall_at_k(gt, gt, 2) == 1.0


def test_timestamped_output_path():
    now = datetime(2026, 3, 4, 5, 6, 7, tzinfo=timezone.utc)
    assert ib._timestamped_output_path(Path("/x/results.csv"), now) == Path("/x/results_20260304_050607.csv")


def test_load_npy_dataset(tmp_path):
    X = np.arange(40, dtype=np.float64).reshape(10, 4)
    np.save(tmp_path / "train.npy", X)
    tr, q, gt = ib._load_npy_dataset(str(tmp_path), num_queries=3)
    assert tr.dtype == np.float32 and tr.shape == (7, 4) and q.shape == (3, 4) and gt is None
    assert np.array_equal(q, X[-3:].astype(np.float32))
    np.save(tmp_path / "queries.npy", X[:2])
    np.save(tmp_path / "ground_truth.npy", np.zeros((2, 5), np.int64))
    tr, q, gt = ib._load_npy_dataset(str(tmp_path), num_queries=3)
    assert tr.shape == (10, 4) and q.shape == (2, 4) and gt.shape == (2, 5)


def test_methods_outside_the_build_are_skipped(tmp_path, capsys):
    rng = np.random.default_rng(0)
    np.save(tmp_path / "train.npy", rng.standard_normal((50, 8)).astype(np.float32))
    np.save(tmp_path / "queries.npy", rng.standard_normal((4, 8)).astype(np.float32))
    np.save(tmp_path / "ground_truth.npy", np.zeros((4, 10), np.int64))  # no GPU call for the GT
    out = ib.ivf_benchmark(dataset=str(tmp_path), methods="saq,rabitq_ivf,nope", bpd=4, k=10, nlist=8, nprobe=2,
                           output=str(tmp_path / "r.csv"), num_queries=4, gt_k=10)
    assert out is None and not list(tmp_path.glob("r_*.csv"))
    text = capsys.readouterr().out
    assert "'saq' is not part of the MI355X build" in text and "'nope' is unknown" in text


def test_cli_registers_ivf_bench():
    from haag_vq.cli import app

    r = CliRunner().invoke(app, ["ivf-bench", "--help"])
    assert r.exit_code == 0 and "--nprobe" in r.output and "--gt-k" in r.output
