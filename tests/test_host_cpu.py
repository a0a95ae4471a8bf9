"""Host logic that needs no GPU: registry dispatch, shard ranges, recall helpers, the run log,
and the multi-rank top-k exchange over gloo (world size 2, CPU tensors).

Mirrors the reference's tests/test_method_registry.py, tests/test_exact_search.py and the
run-log schema of src/haag_vq/utils/run_logger.py:71-115.
"""

import json
import os
import socket
import sqlite3

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from haag_vq.benchmarks import method_registry as reg
from haag_vq.benchmarks.exact_search import recall_at_ks
from haag_vq.metrics.recall import recall_at_k
from haag_vq.parallel import sharded
from haag_vq.utils.run_logger import log_run


def test_largest_divisor_leq():  # reference tests/test_method_registry.py:11-15
    assert reg.largest_divisor_leq(1536, 1536) == 1536
    assert reg.largest_divisor_leq(1536, 600) == 512
    assert reg.largest_divisor_leq(1536, 1) == 1
    assert reg.largest_divisor_leq(30, 7) == 6


def test_method_sets_match_reference():
    assert set(reg.FAISS_METHODS) == {"pq", "opq", "sq"}
    assert set(reg.ALL_METHODS) >= {"pq", "opq", "sq", "saq_paper", "ours", "rabitq", "lvq", "rankaware", "perdim_mse"}


def test_pq_subquantizer_rule():
    # M = largest divisor of D <= round(bpd*D)/8 (method_registry.py:25-28)
    assert reg._pq_subquantizers(1.0, 1536) == 192
    assert reg._pq_subquantizers(4.0, 48) == 24
    assert reg._pq_subquantizers(0.01, 48) == 1


def test_unknown_and_out_of_scope_methods_raise_value_error():
    with pytest.raises(ValueError):
        reg.build_quantizer("bogus", bpd=4, D=48)
    with pytest.raises(ValueError):
        reg.build_quantizer("saq_paper", bpd=4, D=48)


def test_registry_builds_objects_without_gpu():
    # construction is host-only; only fit/compress touch the device
    for m in ("pq", "opq", "sq", "rabitq"):
        assert reg.build_quantizer(m, bpd=4, D=48) is not None


def test_shard_range_covers_rows_once():
    for n in (0, 1, 7, 1000, 1_000_003):
        for world in (1, 2, 3, 8):
            spans = [sharded.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a <= b for a, b in spans)
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def test_recall_helpers():
    gt = np.array([[0, 1, 2, 3], [4, 5, 6, 7]])
    ret = np.array([[0, 9, 2, 8], [7, 6, 5, 4]])
    assert recall_at_k(gt, ret, 2) == pytest.approx((0.5 + 0.0) / 2)
    assert recall_at_k(gt, ret, 4) == pytest.approx((0.5 + 1.0) / 2)
    r = recall_at_ks(ret, gt, ks=(1, 4))
    assert r[1] == pytest.approx(0.5) and r[4] == pytest.approx(0.75)


def test_run_log_schema(tmp_path):
    db = tmp_path / "runs.db"
    log_run("pq", "dummy", {"recall@10": np.float64(0.5), "codes": np.arange(3)}, {"M": 16}, sweep_id="s1",
            db_path=str(db))
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("PRAGMA table_info(runs)")]
    assert cols == ["id", "timestamp", "git_branch", "git_commit", "package_version", "method", "dataset",
                    "cli_command", "metrics_json", "config_json", "sweep_id"]
    method, metrics, cfg, sweep = con.execute("SELECT method, metrics_json, config_json, sweep_id FROM runs").fetchone()
    assert method == "pq" and sweep == "s1"
    assert json.loads(metrics) == {"recall@10": 0.5, "codes": [0, 1, 2]}
    assert json.loads(cfg)["M"] == 16


# ------------------------------------------------------------- gloo exchange (world 2)

def _np_merge(gd, gi, k):
    """Reference merge for the test: (dist, id) order over all parts (NaN after +inf)."""
    P, nq, _ = gd.shape
    d = gd.permute(1, 0, 2).reshape(nq, -1).numpy()
    i = gi.permute(1, 0, 2).reshape(nq, -1).numpy().astype(np.int64) & 0xFFFFFFFF
    dd = np.where(np.isnan(d), np.inf, d)
    out_d = np.empty((nq, k), np.float32)
    out_i = np.empty((nq, k), np.int64)
    for q in range(nq):
        order = np.lexsort((i[q], dd[q]))[:k]
        out_d[q], out_i[q] = d[q, order], i[q, order]
    return torch.from_numpy(out_d), torch.from_numpy(out_i.astype(np.uint32).view(np.int32))


def _worker(rank, world, port, X, Q, k, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b = sharded.shard_range(X.shape[0], rank, world)
        d2 = ((Q[:, None, :] - X[None, a:b, :]) ** 2).sum(-1)  # exact fp64 distances of the shard
        kk = min(k, b - a)
        order = np.lexsort((np.broadcast_to(np.arange(b - a), d2.shape), d2))[:, :kk]
        ld = np.take_along_axis(d2, order, 1).astype(np.float32)
        li = (order + a).astype(np.uint32)
        if kk < k:  # pad like the device kernels: +inf / NO_ID
            ld = np.pad(ld, ((0, 0), (0, k - kk)), constant_values=np.inf)
            li = np.pad(li, ((0, 0), (0, k - kk)), constant_values=0xFFFFFFFF)
        gd, gi = sharded.exchange_topk(torch.from_numpy(ld), torch.from_numpy(li.view(np.int32)), k, merge=_np_merge)
        if rank == 0:
            out.put((gd.numpy(), gi.numpy().view(np.uint32)))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _exchange(X, Q, k, world):
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, X, Q, k, out)) for r in range(world)]
    for p in procs:
        p.start()
    gd, gi = out.get(timeout=240)
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    return gd, gi


def _single_rank(X, Q, k):
    d2 = ((Q[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    ref = np.lexsort((np.broadcast_to(np.arange(X.shape[0]), d2.shape), d2))[:, :k]
    return np.take_along_axis(d2, ref, 1).astype(np.float32), ref


@pytest.mark.parametrize("world", [2, 8])
def test_exchange_topk_gloo_matches_single_rank(world):
    """world 8 = the node's GPU count; gloo stands in for RCCL on CPU tensors."""
    rng = np.random.default_rng(3)
    X = rng.standard_normal((501, 16))
    Q = rng.standard_normal((7, 16))
    k = 10
    gd, gi = _exchange(X, Q, k, world)
    rd, ri = _single_rank(X, Q, k)
    np.testing.assert_array_equal(gi.astype(np.int64), ri)
    np.testing.assert_allclose(gd, rd, rtol=0, atol=0)


def test_exchange_topk_gloo_world8_ties_across_shards():
    """Every database row repeated in all 8 shards: each query's nearest distances occur once per
    shard, so the merged top-k must take the (dist, id) order of mivq_topk_merge — equal
    distances by increasing global id — exactly as one rank over all rows would."""
    rng = np.random.default_rng(11)
    base = rng.standard_normal((63, 8))
    X = np.tile(base, (8, 1))  # shard r (63 rows at world 8) holds a copy of every base row
    Q = rng.standard_normal((5, 8))
    k = 20
    gd, gi = _exchange(X, Q, k, 8)
    rd, ri = _single_rank(X, Q, k)
    np.testing.assert_array_equal(gi.astype(np.int64), ri)
    np.testing.assert_array_equal(gd, rd)
    # the first 8 entries of each query are one base row's 8 copies, in increasing id order
    assert np.all(ri[:, :8] % 63 == ri[:, :1] % 63)
    assert np.all(np.diff(ri[:, :8], axis=1) == 63)
