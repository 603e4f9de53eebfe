#!/usr/bin/env python3
"""Per-dispatch listing of the last N kernels of a rocprofv3 kernel-trace CSV (one bench step):
order, short name, grid, duration and gap to the previous dispatch's end, in microseconds.
    python scripts/step_trace.py <run_kernel_trace.csv> [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"]]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = rows[-n:]


def short(name):
    name = name.replace("void ", "").replace("tq::(anonymous namespace)::", "").replace("tq::", "")
    depth, out = 0, ""
    for ch in name:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out += ch
    return out[:60]


prev_end = None
tot = 0.0
for i, r in enumerate(rows):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    tot += (e - s) / 1e3
    grid = r.get("Grid_Size", r.get("Grid_Size_X", ""))
    print(f"{i:3d} {short(r['Kernel_Name']):60s} grid={grid:>8s} {(e - s) / 1e3:9.1f} us  gap {gap:6.1f}")
    prev_end = e
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"busy {tot:.1f} us of span {span:.1f} us")
