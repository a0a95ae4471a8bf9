"""Multi-rank paths on one GPU (VERDICT r4 "put config #5 behind the product's own
caller"): two ranks share the card and exchange over gloo on host copies.  The RCCL path is the
same code with backend "nccl" (bench.py --gpus N).

* `vq-benchmark streaming-sweep --gpus 2`: the logged MSE / counts equal the single-process run
  bit for bit, and the row carries n_gpus / device / roofline_frac.
* ShardedFlatIndex: the global top-k of two row shards equals the single-device ranking of the
  whole database (ids and distances), L2 and IP, k = 10 and k = 300, with exact duplicates
  across the shard boundary.
"""
import json
import os
import sqlite3
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "vector-quantization_amd"


def _env():
    return dict(os.environ, PYTHONPATH=str(PKG), VQ_DIST_BACKEND="gloo", OMP_NUM_THREADS="1",
                HSA_ENABLE_IPC_MODE_LEGACY="0")


def _rows(db):
    con = sqlite3.connect(db)
    rows = con.execute("SELECT metrics_json, config_json, sweep_id FROM runs").fetchall()
    con.close()
    return [(json.loads(m), json.loads(c), s) for m, c, s in rows]


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["pq", "opq", "sq"])
def test_streaming_sweep_two_ranks_one_gpu(dev, tmp_path, method):
    X = np.random.default_rng(9).standard_normal((20003, 128)).astype(np.float32)
    f = tmp_path / "stream.npy"
    np.save(f, X)
    out = {}
    for g in (1, 2):
        db = tmp_path / f"runs{g}.db"
        cmd = [sys.executable, "-u", "-m", "haag_vq", "streaming-sweep", "--method", method, "--pq-subquantizers", "8",
               "--opq-quantizers", "8", "--training-size", "8192", "--batch-size", "3000", "--data-path", str(f),
               "--db-path", str(db), "--gpus", str(g)]
        p = subprocess.run(cmd, capture_output=True, text=True, env=_env(), timeout=300, cwd=str(tmp_path))
        assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
        rows = _rows(db)
        assert len(rows) == 1  # rank 0 logs the run once
        out[g] = rows[0]
    (m1, c1, _), (m2, c2, _) = out[1], out[2]
    assert m1["total_vectors_compressed"] == m2["total_vectors_compressed"] == 20003
    assert m1["num_batches"] == m2["num_batches"] == 7
    assert m1["mse"] == m2["mse"]  # bit for bit
    assert m1["n_gpus"] == 1 and m2["n_gpus"] == 2 and c1 == c2  # the reference's config
    if method != "sq":
        assert c1 == {"M": 8, "B": 8}
    for m in (m1, m2):
        assert m["device"] and 0.0 < m["roofline_frac"] < 1.0 and m["encode_vectors_per_s"] > 0


@pytest.mark.gpu
def test_sharded_flat_index_two_ranks_one_gpu(dev, tmp_path):
    res_file = tmp_path / "res.json"
    from haag_vq.parallel.launch import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(ROOT / "tests" / "_sharded_worker.py"),
           str(res_file)]
    p = subprocess.run(cmd, capture_output=True, text=True, env=_env(), timeout=300, cwd=str(tmp_path))
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    res = json.loads(res_file.read_text())
    assert res["world"] == 2
    for metric in ("l2", "ip"):
        r = res[metric]
        assert r["sharded_ids"] == r["single_ids"], metric
        assert np.array_equal(np.array(r["sharded_d"], np.float32), np.array(r["single_d"], np.float32)), metric
        assert r["k300_ids"] == r["k300_single_ids"], metric
        assert r["reload_equal"], metric  # save / load of the per-rank shard files
    assert res["l2"]["sharded_ids"][0][:3] == [5, 17, 30008]  # exact duplicates: by id across the shards


@pytest.mark.gpu
def test_sweep_logs_device_fields(dev, tmp_path):
    from haag_vq.benchmarks.sweep import sweep

    db = tmp_path / "s.db"
    sweep(method="sq", dataset="dummy", num_samples=2000, dim=64, dataset_limit=None, cache_dir=str(tmp_path),
          pq_subquantizers="8", pq_bits="8", sq_bits="8", rabitq_metric_type="L2", saq_num_bits="4",
          saq_total_bits="", saq_allowed_bits="", saq_segments="", opq_quantizers="8", opq_bits="8",
          with_recall=False, with_pairwise=False, with_rank=False, num_pairs=10, rank_k=10, ground_truth_path=None,
          codebooks_dir=str(tmp_path / "cb"), db_path=str(db), gpus=1, device=None)
    (m, c, _), = _rows(db)
    assert m["n_gpus"] == 1 and m["device"] and "n_gpus" not in c  # config_json: the reference's grid config
    assert m["encode_device_ms"] > 0 and 0.0 < m["roofline_frac"] < 1.0


@pytest.mark.gpu
def test_sweep_two_ranks_deal_configs(dev, tmp_path):
    """`vq-benchmark sweep --gpus 2`: the grid's configurations go to the ranks round-robin, every
    configuration is logged once under one sweep id, and each row equals the single-process
    run of the same configuration (codes and metrics are deterministic)."""
    base = [sys.executable, "-u", "-m", "haag_vq", "sweep", "--method", "pq", "--dataset", "dummy",
            "--num-samples", "3000", "--dim", "64", "--pq-subquantizers", "4,8,16", "--pq-bits", "8",
            "--no-with-recall", "--no-with-pairwise", "--no-with-rank", "--codebooks-dir", str(tmp_path / "cb")]
    out = {}
    for g in (1, 2):
        db = tmp_path / f"sweep{g}.db"
        p = subprocess.run(base + ["--db-path", str(db), "--gpus", str(g)], capture_output=True, text=True,
                           env=_env(), timeout=300, cwd=str(tmp_path))
        assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
        out[g] = _rows(db)
    assert len(out[1]) == len(out[2]) == 3
    assert len({sid for _, _, sid in out[2]}) == 1  # one sweep id across the ranks
    one = {c["subquantizers"]: m for m, c, _ in out[1]}
    two = {c["subquantizers"]: m for m, c, _ in out[2]}
    assert set(one) == set(two) == {4, 8, 16}
    for M in one:
        assert two[M]["n_gpus"] == 2 and one[M]["n_gpus"] == 1
        assert two[M]["reconstruction_distortion"] == one[M]["reconstruction_distortion"]
        assert two[M]["compression_ratio"] == one[M]["compression_ratio"]


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu(dev, tmp_path):
    """`bench.py --gpus 2` end to end on one card (VQ_DIST_BACKEND=gloo: host-staged
    collectives instead of RCCL): the launcher, per-rank shards, the codebook and query
    broadcasts, max-over-ranks timing, the top-k exchange and merge, config #5 -- the code the
    driver's multi-GPU runs execute, with small shapes.  The sharded ADC lists must agree with
    the sharded decode + exact ranking of the same codes (near-ties aside)."""
    cmd = [sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", "2", "--n", "100000", "--steps", "2",
           "--warmup", "1", "--nq", "64", "--gt-queries", "32", "--no-cpu-baseline", "--no-alt-data",
           "--no-north-star", "--no-configs", "--config5-rows", "60000", "--config5-nq", "64"]
    p = subprocess.run(cmd, capture_output=True, text=True, env=_env(), timeout=600, cwd=str(tmp_path))
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, p.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["config"]["parallelism"] == "row-sharded x2"
    assert out["adc"]["n_total"] == 200000 and out["adc"]["topk_agreement_adc_vs_decode_exact"] >= 0.99
    c5 = out["config5"]
    assert c5["n_gpus"] == 2 and c5["rows_total"] == 120000 and c5["adc"]["topk_agreement_adc_vs_decode_exact"] >= 0.99


@pytest.mark.gpu
def test_rccl_collectives_world1(dev, tmp_path):
    """RCCL on the hardware: an "nccl" process group of world size 1 on the card runs every
    collective the multi-GPU path issues (broadcast, broadcast_object_list, all_gather_into_tensor
    + mivq_topk_merge, all_reduce MAX) on device tensors; each must return its input.  Two ranks
    cannot share one GPU under RCCL, so the multi-rank tests above use gloo."""
    from haag_vq.parallel.launch import free_port

    res_file = tmp_path / "rccl.json"
    env = dict(os.environ, PYTHONPATH=str(PKG), HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(free_port()), RANK="0", LOCAL_RANK="0", WORLD_SIZE="1")
    env.pop("VQ_DIST_BACKEND", None)
    p = subprocess.run([sys.executable, "-u", str(ROOT / "tests" / "_rccl_worker.py"), str(res_file)],
                       capture_output=True, text=True, env=env, timeout=180, cwd=str(tmp_path))
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    res = json.loads(res_file.read_text())
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["broadcast_equal"] and res["object_equal"] and res["allgather_merge_equal"]
    assert res["sizes"] == [123457] and res["allreduce_max"] == 1.25
