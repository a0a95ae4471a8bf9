"""Summarise rocprofv3 --pmc passes for one kernel: per-dispatch averages of each counter.

usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> <kernel-substring> [last_n]
(last_n: only the last N dispatches of each pass among those with the kernel's largest grid,
tools/pmc_select.py -- the benched full-size call, never a smaller launch of the same kernel)
Prints counters and the derived HBM traffic (gfx950: FETCH_SIZE reads half the bytes of a
wide coalesced stream -> x2, MI355X_MICROARCH.md §HBM; FETCH/WRITE_SIZE are in KiB).
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_select import select  # noqa: E402

root, sub = sys.argv[1], sys.argv[2]
last_n = int(sys.argv[3]) if len(sys.argv) > 3 else None
vals, durs, grid = select(root, sub, last_n)
print(f"(dispatches with grid size {grid}: the largest launch of this kernel in the run)")
out = {k: sum(v) / len(v) for k, v in vals.items()}
for k, v in sorted(out.items()):
    print(f"{k:28s} {v:16.1f}  (n={len(vals[k])})")
if "FETCH_SIZE" in out:
    rd = out["FETCH_SIZE"] * 1024 * 2
    wr = out.get("WRITE_SIZE", 0.0) * 1024
    print(f"HBM read (corrected x2) {rd/1e9:.3f} GB/launch, write {wr/1e9:.4f} GB/launch, total {(rd+wr)/1e9:.3f} GB")
    out["hbm_bytes_per_launch"] = rd + wr
print(json.dumps(out))
