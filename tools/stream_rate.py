"""Device encode rate of `vq-benchmark streaming-sweep` (BASELINE config #5's caller,
/root/reference/src/haag_vq/benchmarks/streaming_sweep.py:153-185) at its default 10,000-row
batches, against the same codebook's device-resident single-call rate.

usage: python tools/stream_rate.py [--n 2000000] [--d 1024] [--M 16] [--batch-size 10000]

Writes an (n, d) unit-normalised Gaussian .npy (seed 0) under $TMPDIR, runs the CLI command
in-process twice -- grouped device calls (the product default, streaming_sweep.CALL_ROWS) and
one call per stream batch (upstream's loop) -- and prints each run's logged
encode_vectors_per_s / roofline_frac / MSE, then the rate of one device-resident call over
the same rows with the same quantizer (the bench's config5 leg measures that kind of call).
"""
import argparse
import json
import os
import sqlite3
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_000_000)
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--batch-size", type=int, default=10_000)
    ap.add_argument("--training-size", type=int, default=65_536)
    a = ap.parse_args()
    import torch
    from typer.testing import CliRunner

    from haag_vq import _native
    from haag_vq.benchmarks import streaming_sweep as ss
    from haag_vq.cli import app

    tmp = Path(tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp")))
    f = tmp / "stream.npy"
    t0 = time.time()
    rng = np.random.default_rng(0)
    X = np.lib.format.open_memmap(f, mode="w+", dtype=np.float32, shape=(a.n, a.d))
    for s in range(0, a.n, 262_144):
        blk = rng.standard_normal((min(262_144, a.n - s), a.d), dtype=np.float32)
        blk /= np.linalg.norm(blk, axis=1, keepdims=True)
        X[s:s + blk.shape[0]] = blk
    X.flush()
    del X
    print(f"wrote {f} ({a.n} x {a.d}) in {time.time() - t0:.1f} s", flush=True)
    res = {}
    for tag, rows in (("grouped", ss.CALL_ROWS), ("per_batch", a.batch_size)):
        ss.CALL_ROWS = rows
        db = tmp / f"{tag}.db"
        t0 = time.time()
        out = CliRunner().invoke(app, ["streaming-sweep", "--method", "pq", "--pq-subquantizers", str(a.M),
                                       "--training-size", str(a.training_size), "--batch-size", str(a.batch_size),
                                       "--data-path", str(f), "--db-path", str(db)])
        wall = time.time() - t0
        if out.exit_code != 0:
            print(out.output[-3000:], repr(out.exception), flush=True)
            sys.exit(1)
        con = sqlite3.connect(db)
        (mj,), = con.execute("SELECT metrics_json FROM runs").fetchall()
        con.close()
        m = json.loads(mj)
        res[tag] = m
        print(json.dumps({"run": tag, "rows_per_call": min(rows, a.n), "wall_s": round(wall, 2),
                          "encode_device_s": m["encode_device_s"], "encode_vectors_per_s": m["encode_vectors_per_s"],
                          "roofline_frac": m["roofline_frac"], "mse": m["mse"], "num_batches": m["num_batches"]}),
              flush=True)
    same = res["grouped"]["mse"] == res["per_batch"]["mse"]
    # the same rows as one device-resident call (as the bench's config5 leg), same codebook recipe
    from haag_vq.methods.product_quantization import ProductQuantizer

    Xm = np.load(f, mmap_mode="r")
    pq = ProductQuantizer(M=a.M, B=8)
    pq.fit(np.ascontiguousarray(Xm[:a.training_size]))
    Xd = torch.from_numpy(np.ascontiguousarray(Xm)).cuda()
    C = pq.centroids_device
    prep = _native.pq_prepare(C, 8)
    for _ in range(3):
        _native.pq_encode(Xd, C, prep, 8)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _native.pq_encode(Xd, C, prep, 8)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3)
    t = sorted(ts)[len(ts) // 2]
    rate = a.n / t
    print(json.dumps({"run": "device_resident_one_call", "rows": a.n, "median_s": t, "vectors_per_s": rate,
                      "roofline_frac": a.n * (4 * a.d + a.M) / t / 8e12}), flush=True)
    print(json.dumps({"grouped_over_device_call": res["grouped"]["encode_vectors_per_s"] / rate,
                      "per_batch_over_device_call": res["per_batch"]["encode_vectors_per_s"] / rate,
                      "mse_identical": same}), flush=True)
    f.unlink()
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
