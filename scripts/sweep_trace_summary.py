#!/usr/bin/env python3
"""Summarise sweep2 launches of a rocprofv3 kernel trace: the per-slice big launch (> 100 us) and
the total sweep2 time per execute.  usage: sweep_trace_summary.py <trace.csv> <label> [n_exec]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n_exec = int(sys.argv[3]) if len(sys.argv) > 3 else 4
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "sweep2" in r["Kernel_Name"]]
big = sorted(x for x in d if x > 100)
med = big[len(big) // 2] if big else 0
print(f"{sys.argv[2]}: sweep2 launches {len(d)}, big {len(big)} median {med:.1f} us min {big[0] if big else 0:.1f}, "
      f"sweep2 total per execute {sum(d) / n_exec:.1f} us")
