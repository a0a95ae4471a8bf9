"""Generate the committed golden fixtures from the REFERENCE implementation.

Run in the build container only (it imports /root/reference/src, which does not exist
on the GPU box):

    python tests/golden/make_golden.py

Outputs (all small, compressed, data only):
  sq_golden.npz        inputs / lo / hi / codes / reconstructions produced by the
                       reference's ScalarQuantizer (scalar_quantization.py:37-90) for
                       bits 4/8/16, fp32 and fp64 inputs, odd/even D, and inputs
                       outside the fitted range (numpy's wrap-around cast).
  extrabitq_golden.npz model state + codes + reconstructions of the reference's
                       ExtendedRaBitQuantizer (extended_rabitq.py:47-199).
  kat.json             the known-answer rows of logs/benchmark_runs.db (ids 38, 52,
                       56, 46-48) read through sqlite3 in read-only mode.
"""

from __future__ import annotations

import json
import sqlite3
import sys
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent


def _import_reference():
    sys.path.insert(0, str(REF / "src"))
    from haag_vq.methods.scalar_quantization import ScalarQuantizer  # noqa: E402
    from haag_vq.methods.extended_rabitq import ExtendedRaBitQuantizer  # noqa: E402
    return ScalarQuantizer, ExtendedRaBitQuantizer


def make_sq(ScalarQuantizer) -> None:
    arrays = {}
    cases = []
    rng = np.random.default_rng(7)
    for dtype in (np.float32, np.float64):
        for d in (7, 64, 130):
            for bits in (4, 8, 16):
                tag = f"{np.dtype(dtype).name}_d{d}_b{bits}"
                X = (rng.standard_normal((130, d)) * rng.uniform(0.1, 3.0, d)).astype(dtype)
                q = ScalarQuantizer(num_bits=bits)
                q.fit(X[:100])                      # fit on a subset ...
                codes = q.compress(X)               # ... so rows 100+ leave the range
                recon = q.decompress(codes)
                arrays[f"{tag}_X"] = X
                arrays[f"{tag}_lo"] = q.min
                arrays[f"{tag}_hi"] = q.max
                arrays[f"{tag}_codes"] = codes
                arrays[f"{tag}_recon"] = recon
                cases.append(tag)
    arrays["cases"] = np.array(cases)
    np.savez_compressed(OUT / "sq_golden.npz", **arrays)


def make_extrabitq(ExtendedRaBitQuantizer) -> None:
    arrays = {}
    cases = []
    rng = np.random.default_rng(11)
    X = rng.standard_normal((200, 64)).astype(np.float32)
    for bits in (1, 2, 4, 8):
        q = ExtendedRaBitQuantizer(num_bits=bits, seed=0)
        q.fit(X)
        codes = q.compress(X)
        tag = f"b{bits}"
        arrays[f"{tag}_c"] = q.c
        arrays[f"{tag}_P"] = q.P
        arrays[f"{tag}_levels"] = q.levels
        arrays[f"{tag}_codes"] = codes
        arrays[f"{tag}_recon"] = q.decompress(codes)
        cases.append(tag)
    arrays["X"] = X
    arrays["cases"] = np.array(cases)
    np.savez_compressed(OUT / "extrabitq_golden.npz", **arrays)


def make_kat() -> None:
    con = sqlite3.connect(f"file:{REF / 'logs' / 'benchmark_runs.db'}?mode=ro", uri=True)
    rows = {}
    for rid, method, dataset, cli, metrics, config in con.execute(
        "SELECT id, method, dataset, cli_command, metrics_json, config_json FROM runs "
        "WHERE id IN (38, 46, 47, 48, 49, 52, 56)"
    ):
        rows[str(rid)] = {
            "method": method,
            "dataset": dataset,
            "cli_command": cli,
            "metrics": json.loads(metrics),
            "config": json.loads(config) if config else {},
        }
    con.close()
    (OUT / "kat.json").write_text(json.dumps(rows, indent=1, sort_keys=True) + "\n")


def main() -> None:
    ScalarQuantizer, ExtendedRaBitQuantizer = _import_reference()
    make_sq(ScalarQuantizer)
    make_extrabitq(ExtendedRaBitQuantizer)
    make_kat()
    print("wrote", sorted(p.name for p in OUT.iterdir() if p.suffix in (".npz", ".json")))


if __name__ == "__main__":
    main()
