"""Median duration per distinct kernel instance (full template name) in a rocprofv3 kernel
trace: python tools/ktrace_v.py <trace.csv> <substr>"""
import csv
import re
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2]
d = defaultdict(list)
for r in rows:
    if sub in r["Kernel_Name"]:
        d[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (k, g), v in sorted(d.items()):
    short = re.sub(r"^void ", "", k.replace("(anonymous namespace)::", "")).split("(")[0]
    short = re.sub(r"^_ZN4mivq12_GLOBAL__N_1\d+", "", short).replace("mivq::", "")[:60]
    print(f"{short:60s} grid {g:8d} n={len(v):3d} median {statistics.median(v):8.1f} us  min {min(v):8.1f}")
