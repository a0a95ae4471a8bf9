"""Write profiles/traffic.json: HBM bytes per mivq_pq_encode call from a tools/pmc.sh run.

usage: python tools/traffic.py gpurun_out/pmc_<tag> <workload> [last_n]
Sums the per-launch HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, gfx950 corrections as in
tools/pmc_summary.py) of the four kernels of one encode call.
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

KERNELS = ("pq_encode_cs_kernel", "pq_resolve_merged", "pq_transpose_codes")


def per_launch(root, sub, last_n):
    vals = defaultdict(list)
    for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
        rows = [r for r in csv.DictReader(open(f)) if sub in r["Kernel_Name"]]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})[-last_n:]
        for r in rows:
            if int(r["Dispatch_Id"]) in ids and r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    fetch = sum(vals["FETCH_SIZE"]) / max(1, len(vals["FETCH_SIZE"]))
    write = sum(vals["WRITE_SIZE"]) / max(1, len(vals["WRITE_SIZE"]))
    return fetch * 1024 * 2 + write * 1024


def main():
    root, workload = sys.argv[1], sys.argv[2]
    last_n = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    parts = {k: per_launch(root, k, last_n) for k in KERNELS}
    out_path = Path(__file__).resolve().parent.parent / "profiles" / "traffic.json"
    data = json.loads(out_path.read_text()) if out_path.exists() else {}
    data[workload] = {"bytes_per_launch": sum(parts.values()), "per_kernel": parts,
                      "source": f"{root} (rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE, FETCH x2 gfx950 correction, KiB)"}
    out_path.write_text(json.dumps(data, indent=1) + "\n")
    print(json.dumps(data[workload], indent=1))


if __name__ == "__main__":
    main()
