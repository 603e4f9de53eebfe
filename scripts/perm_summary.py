#!/usr/bin/env python3
"""Summarise permute_bench.py logs and the permute PMC passes (FETCH_SIZE x2 per the gfx950
correction, WRITE_SIZE; KB units) into one table.  usage: perm_summary.py <bench.log>... [--pmc DIR]"""
import collections
import csv
import json
import os
import sys


def bench(paths):
    for p in paths:
        print(p)
        for line in open(p):
            if line.startswith("{"):
                d = json.loads(line)
                kind = d["plan"].split("[")[-1].split("]")[0]
                print(f"  {d['dtype']:5s} rank {d['rank']:2d} {kind:8s} {d['avg_launch_ms']*1e3:8.1f} us "
                      f"{d['GBps']:7.0f} GB/s frac {d['frac']:.3f} exact {d['bit_exact']}")


def pmc(root):
    agg = collections.defaultdict(dict)
    for sub in ("pmcpf", "pmcpw", "pmcps"):
        f = os.path.join(root, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = (sub, int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0][-60:])
            agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k in sorted(agg):
        print(k, {a: round(b) for a, b in agg[k].items()})


if __name__ == "__main__":
    args = sys.argv[1:]
    if "--pmc" in args:
        i = args.index("--pmc")
        pmc(args[i + 1])
        args = args[:i] + args[i + 2:]
    bench(args)
