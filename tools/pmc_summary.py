"""Summarise rocprofv3 --pmc passes for one kernel: per-dispatch averages of each counter.

usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> <kernel-substring> [last_n]
(last_n: only the last N matching dispatches of each pass, e.g. the timed bench steps)
Prints counters and the derived HBM traffic (gfx950: FETCH_SIZE reads half the bytes of a
wide coalesced stream -> x2, MI355X_MICROARCH.md §HBM; FETCH/WRITE_SIZE are in KiB).
"""
import csv
import glob
import json
import sys
from collections import defaultdict

root, sub = sys.argv[1], sys.argv[2]
last_n = int(sys.argv[3]) if len(sys.argv) > 3 else None
vals = defaultdict(list)
durs = []
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    rows = [r for r in csv.DictReader(open(f)) if sub in r["Kernel_Name"]]
    if last_n is not None:
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})[-last_n:]
        rows = [r for r in rows if int(r["Dispatch_Id"]) in ids]
    for r in rows:
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = {k: sum(v) / len(v) for k, v in vals.items()}
for k, v in sorted(out.items()):
    print(f"{k:28s} {v:16.1f}  (n={len(vals[k])})")
if "FETCH_SIZE" in out:
    rd = out["FETCH_SIZE"] * 1024 * 2
    wr = out.get("WRITE_SIZE", 0.0) * 1024
    print(f"HBM read (corrected x2) {rd/1e9:.3f} GB/launch, write {wr/1e9:.4f} GB/launch, total {(rd+wr)/1e9:.3f} GB")
    out["hbm_bytes_per_launch"] = rd + wr
print(json.dumps(out))
