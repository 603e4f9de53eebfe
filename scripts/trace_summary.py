#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace CSV: per-kernel-name totals, and (with --last N) the
busy/idle split of the last N dispatches (sum of kernel durations vs their start..end span)."""
import argparse, csv, collections, re

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--last", type=int, default=0)
args = ap.parse_args()
rows = list(csv.DictReader(open(args.csv)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"]]
if args.last:
    rows = rows[-args.last:]


def short(n):
    n = n.replace("void ", "").replace("tq::(anonymous namespace)::", "").replace("tq::", "")
    depth, out = 0, ""
    for ch in n:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out += ch
    return out


tot = collections.defaultdict(lambda: [0, 0])
busy = 0
for r in rows:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    k = short(r["Kernel_Name"])
    tot[k][0] += 1
    tot[k][1] += d
    busy += d
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
print(f"kernels {len(rows)} busy {busy/1e6:.3f} ms span {span/1e6:.3f} ms")
for k, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{d/1e6:10.3f} ms {n:7d} x {d/max(1,n)/1e3:9.2f} us  {k}")
