"""CPU: the measurement tools' selection logic (tools/pmc_select.py) on synthetic rocprofv3
counter CSVs -- a PMC summary must describe the benched launch, not a smaller one of the same
kernel (round-3 VERDICT: the OPQ32 entry averaged two 1000-query rotations with a 1M one)."""

import csv
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))


def _write(path, rows):
    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name",
                                          "Counter_Value", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _row(i, grid, val, name="opq_split_gemm_kernel<2, 2, 4, 4>", counter="SQ_INSTS_MFMA"):
    return {"Dispatch_Id": i, "Grid_Size": grid, "Kernel_Name": name, "Counter_Name": counter,
            "Counter_Value": val, "Start_Timestamp": 0, "End_Timestamp": 1000}


def test_select_takes_the_largest_grid(tmp_path):
    from pmc_select import select

    big, small = 3_000_000, 3_000
    # the timed 1M rotations, then the search's 1000-query rotations, then a 1M reverse rotation
    rows = [_row(1, big, 432e6), _row(2, big, 432e6), _row(3, small, 0.5e6), _row(4, small, 0.5e6),
            _row(5, big, 432e6), _row(6, 10, 1.0, name="other")]
    _write(tmp_path / "p1" / "run_counter_collection.csv", rows)
    vals, durs, grid = select(str(tmp_path), "opq_split_gemm", 3)
    assert grid == big
    assert vals["SQ_INSTS_MFMA"] == [432e6] * 3  # the old "last 3" would have mixed in 2 small ones
    assert len(durs) == 3
    vals, _, grid = select(str(tmp_path), "opq_split_gemm", 3, grid=small)
    assert grid == small and vals["SQ_INSTS_MFMA"] == [0.5e6] * 2


def test_select_per_pass_and_missing(tmp_path):
    from pmc_select import select

    _write(tmp_path / "p1" / "run_counter_collection.csv", [_row(1, 8, 1.0, counter="FETCH_SIZE")])
    _write(tmp_path / "p2" / "run_counter_collection.csv", [_row(1, 8, 2.0, counter="WRITE_SIZE")])
    vals, _, grid = select(str(tmp_path), "opq_split_gemm", 3)
    assert grid == 8 and vals["FETCH_SIZE"] == [1.0] and vals["WRITE_SIZE"] == [2.0]
    assert select(str(tmp_path), "no_such_kernel", 3) == ({}, [], None)


def test_gpurunignore_keeps_what_the_gpu_runs_read():
    """bench.py reads profiles/traffic.json on the GPU box (roofline.traffic); the library and the
    golden fixtures must travel too.  tar --exclude semantics: a pattern matches a member path
    (wildcards match '/'), and excluding a directory excludes everything under it."""
    import fnmatch

    root = Path(__file__).resolve().parents[1]
    pats = [p.strip() for p in (root / ".gpurunignore").read_text().splitlines() if p.strip()]

    def excluded(rel):
        parts = rel.split("/")
        prefixes = ["./" + "/".join(parts[:i]) for i in range(1, len(parts) + 1)]
        for p in pats:
            for cand in prefixes:
                if fnmatch.fnmatch(cand, p) or (not p.startswith("./") and fnmatch.fnmatch(cand.split("/")[-1], p)):
                    return True
        return False

    for rel in ("profiles/traffic.json", "vector-quantization_amd/lib/libmivq.so", "bench.py",
                "tests/golden/sq_golden_wide.npz", "oracle/mivq_oracle.c", "include/mivq.h"):
        assert not excluded(rel), rel
    assert excluded("profiles/r04_s11/bench_default.log")
