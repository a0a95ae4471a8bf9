"""Which dispatches of a kernel a PMC summary averages (shared by tools/traffic.py and
tools/pmc_summary.py).

A bench run launches the same kernel at several sizes (the OPQ32 leg: the 1M x 1536 rotation of
the timed step and of the recall check, but also 1000-query rotations of the search), so "the
last N dispatches" can mix shapes (round-3 VERDICT: the opq32 entry averaged two 1000-query
rotations with one 1M rotation).  Rule: keep the dispatches with the LARGEST grid (the benched
full-size call), then the last N of those; every selected dispatch must have the same grid, or
the selection is refused.
"""
from __future__ import annotations

import csv
import glob
from collections import defaultdict


def _grid(r: dict) -> int:
    for key in ("Grid_Size", "Grid_Size_X", "grid_size"):
        if key in r and r[key] not in (None, ""):
            try:
                return int(float(r[key]))
            except ValueError:
                pass
    return -1


def select(root: str, sub: str, last_n: int | None = 3, grid: int | None = None):
    """{counter: [values of the selected dispatches]}, [durations us], selected grid size.

    sub: kernel-name substring; grid: an explicit grid size to select instead of the largest."""
    rows = []
    for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
        rows += [dict(r, _file=f) for r in csv.DictReader(open(f)) if sub in r["Kernel_Name"]]
    if not rows:
        return {}, [], None
    grids = {_grid(r) for r in rows}
    g = grid if grid is not None else max(grids)
    rows = [r for r in rows if _grid(r) == g]
    vals, durs = defaultdict(list), []
    by_file = defaultdict(list)
    for r in rows:
        by_file[r["_file"]].append(r)
    for f, rs in by_file.items():  # last N dispatches of THIS pass (dispatch ids restart per run)
        ids = sorted({int(r["Dispatch_Id"]) for r in rs})
        if last_n is not None:
            ids = ids[-last_n:]
        keep = set(ids)
        sel = [r for r in rs if int(r["Dispatch_Id"]) in keep]
        if len({_grid(r) for r in sel}) != 1:
            raise SystemExit(f"pmc_select: {sub}: selected dispatches differ in grid size")
        for r in sel:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return vals, durs, g
