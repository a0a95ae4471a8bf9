"""bench.py's multi-rank launcher on CPU (no GPU): `--gpus N` starts torch.distributed.run as a
child process, the ranks exchange per-shard top-k over gloo, and rank 0's merged lists must
equal the single-rank answer (the `--dry-run` rehearsal of the RCCL path)."""

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                       timeout=300, env=env, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_launcher_dry_run(n):
    out = _run("--gpus", str(n), "--dry-run")
    assert out["n_gpus"] == n
    assert out["dry_run"] is True
    assert out["merged_equals_single"] is True
    assert out["config"]["parallelism"] == f"row-sharded x{n}"


def test_gpus_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--dry-run"], capture_output=True,
                       text=True, timeout=120, env=env, cwd=str(ROOT))
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr


def test_launcher_passes_flags_that_abbreviate_torchrun_options():
    """--n / --d abbreviate several torch.distributed.run options (--nnodes, --nproc-per-node,
    --duplicate-*): the launcher ends torchrun's options with "--" so they reach bench.py."""
    out = _run("--gpus", "2", "--dry-run", "--n", "1000", "--d", "64", "--nq", "10")
    assert out["n_gpus"] == 2 and out["merged_equals_single"] is True
