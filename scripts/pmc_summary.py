#!/usr/bin/env python3
"""Average per-dispatch PMC counters of kernels matching a name fragment, over the passes under a
gpurun_out directory (pmc*/run_counter_collection.csv)."""
import collections, csv, glob, sys
frag = sys.argv[1] if len(sys.argv) > 1 else "sweep2"
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
out = {}
for f in sorted(glob.glob(f"{root}/pmc*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        if frag not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"][:48] + " grid=" + r.get("Grid_Size", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        out.setdefault(k, {}).update({c: sum(x) / len(x) for c, x in v.items()})
for k, v in out.items():
    print(k)
    w = v.get("SQ_WAVES", 0)
    for c in sorted(v):
        extra = f"   per wave {v[c] / w:10.1f}" if w and c.startswith("SQ_") and c != "SQ_WAVES" else ""
        print(f"  {c:24s} {v[c]:16.1f}{extra}")
