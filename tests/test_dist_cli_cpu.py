"""CPU tests of the multi-GPU command-line plumbing: `vq-benchmark
streaming-sweep --gpus N` starts N ranks under torch.distributed.run as a child process,
deals the stream's batches to them in contiguous runs and reduces the per-batch values so
that the result is the single-process one bit for bit.  The ranks run over gloo here
(--dry-run: no quantizer, each batch contributes its sum of squares); the GPU run of the same
path is tests/test_sharded_gpu.py."""

import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "vector-quantization_amd"


def _run_cli(*args, timeout=240):
    env = dict(os.environ, PYTHONPATH=str(PKG), OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "-m", "haag_vq", *args], capture_output=True, text=True, env=env,
                       timeout=timeout, cwd=str(ROOT))
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{") and '"dry_run"' in ln]
    assert len(lines) == 1, p.stdout[-3000:]
    return json.loads(lines[0]), p.stdout


def test_batch_plan_partitions_the_stream():
    from haag_vq.benchmarks.streaming_sweep import batch_plan

    for n, bs, mb in ((1003, 100, None), (1003, 100, 7), (50, 100, None), (0, 10, None), (1000, 100, 10)):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                starts, (b0, b1) = batch_plan(n, bs, mb, r, world)
                assert 0 <= b0 <= b1 <= len(starts)
                seen += list(range(b0, b1))
            assert seen == list(range(len(starts)))  # every batch once, in order
            assert starts == list(range(0, n, bs))[:mb] if mb else starts == list(range(0, n, bs))


def test_rank_command_uses_loopback_and_module():
    from haag_vq.parallel.launch import rank_command

    cmd = rank_command(4, ["streaming-sweep", "--gpus", "4"], port=12345)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=12345" in cmd
    assert cmd[-6:] == ["-m", "--", "haag_vq", "streaming-sweep", "--gpus", "4"]


@pytest.mark.parametrize("gpus", [2, 3])
def test_streaming_sweep_ranks_reduce_to_single_process(tmp_path, gpus):
    X = np.random.default_rng(5).standard_normal((1003, 16)).astype(np.float32)
    f = tmp_path / "stream.npy"
    np.save(f, X)
    base = ["streaming-sweep", "--dataset", "t", "--data-path", str(f), "--batch-size", "100", "--dry-run"]
    one, _ = _run_cli(*base)
    many, out = _run_cli(*base, "--gpus", str(gpus))
    assert "[launcher]" in out and "torch.distributed.run" in out
    assert many["world"] == gpus and one["world"] == 1
    assert many["rows"] == one["rows"] == 1003 and many["batches"] == one["batches"] == 11
    assert many["sum_sq"] == one["sum_sq"]  # bit for bit: each batch on one rank, summed in stream order
    ref = 0.0
    for s in range(0, 1003, 100):
        xb = X[s:s + 100].astype(np.float64)
        ref += float((xb * xb).sum())
    assert one["sum_sq"] == ref
    capped, _ = _run_cli(*base, "--gpus", str(gpus), "--max-batches", "4")
    assert capped["batches"] == 4 and capped["rows"] == 400


def test_cli_exposes_gpus_and_device():
    from typer.testing import CliRunner

    from haag_vq.cli import app

    out = CliRunner().invoke(app, ["sweep", "--help"]).output
    assert "--gpus" in out and "--device" in out
    out = CliRunner().invoke(app, ["streaming-sweep", "--help"]).output
    assert "--gpus" in out
