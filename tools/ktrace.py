"""Per-kernel durations from a rocprofv3 --kernel-trace CSV: python tools/ktrace.py <trace.csv> [substr ...]
Prints, per kernel name substring, the dispatch count and the mean / min of the last half of
its dispatches (steady state), in microseconds."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keys = sys.argv[2:] or ["pq_encode_cs_kernel", "pq_resolve", "transpose_codes", "opq_split", "adc_scan"]
for k in keys:
    v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if k in r["Kernel_Name"]]
    if not v:
        continue
    tail = v[len(v) // 2:]
    print(f"{k:28s} n={len(v):3d}  last-half mean {sum(tail) / len(tail):8.1f} us  min {min(tail):8.1f} us  "
          f"all: {' '.join(f'{x:.0f}' for x in v[-8:])}")
