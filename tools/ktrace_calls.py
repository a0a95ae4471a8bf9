"""Per-call split of mivq_pq_encode from a rocprofv3 --kernel-trace CSV, by launch size.

usage: python tools/ktrace_calls.py <run_kernel_trace.csv> [--last N]

Every encode call (or 2^21-row slice of a large call) is the sequence filter
(pq_encode_cs_kernel) -> resolve (pq_resolve_merged_kernel) -> code transpose
(pq_transpose_codes*) on one queue.  The filter's grid does not depend on the row count (a fixed
number of workgroups per subspace), so the rows of a call are read off its transpose launch
(grid = rows rounded up to 256).  Prints, per (filter instance, rows): the number of calls and
the median filter / resolve / transpose durations and their sum, in microseconds; --last N
keeps the last N calls of each group (the timed steps of a bench run).
"""
import argparse
import csv
import re
import statistics
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    n = n.split("(")[0]
    n = re.sub(r"^_ZN4mivq12_GLOBAL__N_1\d+", "", n)
    return n.replace("mivq::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    pend = {}  # queue -> {"filter": (name, us), "resolve": us}
    calls = defaultdict(list)
    for r in rows:
        name, q = r["Kernel_Name"], r["Queue_Id"]
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "pq_encode_cs_kernel" in name:
            pend[q] = {"filter": (short(name), us), "resolve": 0.0}
        elif "pq_resolve_merged_kernel" in name and q in pend:
            pend[q]["resolve"] += us
        elif "pq_transpose_codes" in name and q in pend:
            p = pend.pop(q)
            rows_ = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            calls[(p["filter"][0], rows_)].append((p["filter"][1], p["resolve"], us))
    print(f"{'filter instance':52s} {'rows~':>9s} {'calls':>5s} {'filter':>9s} {'resolve':>8s} {'transp':>7s} {'sum':>9s}  us")
    for (fname, nrows), v in sorted(calls.items(), key=lambda kv: (kv[0][0], kv[0][1])):
        v = v[-a.last:] if a.last else v
        f, rs, t = (statistics.median(x[i] for x in v) for i in range(3))
        print(f"{fname[:52]:52s} {nrows:9d} {len(v):5d} {f:9.1f} {rs:8.1f} {t:7.1f} {f + rs + t:9.1f}")


if __name__ == "__main__":
    main()
