#!/usr/bin/env python3
"""Match a rocprofv3 kernel trace of `rank_sim.py C4 8` (one execute = hoisted + 1 slice) to the
plan's launch schedule and print per-launch duration, ops and algorithmic GB/s."""
import csv, os, re, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tneq_qc_amd  # noqa
from tneq_qc_amd.circuits import config_task
from tneq_qc_amd.expression import HipContractExpression

t = config_task(sys.argv[2] if len(sys.argv) > 2 else "C4")
e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
p = e.plan(torch.complex64)
lines = p.describe().splitlines()
ops = [l for l in lines if not l.startswith("#")]
sched = [[int(x) for x in l.split()[2:]] + [l.split()[1]] for l in lines if l.startswith("# once") or l.startswith("# slice")]
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"] and "splitk" not in r["Kernel_Name"]]
rows = rows[-len(sched):]
tot = {"once": 0.0, "slice": 0.0}
for g, r in zip(sched, rows):
    kind, ids = g[-1], g[:-1]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    by = 0
    for i in ids:
        m = re.search(r"tin=(\d+) tout=(\d+) cols=(\d+)", ops[i])
        if m:
            a, b, c = map(int, m.groups())
            by += (a + b) * c * 8
    tot[kind] += d
    desc = ops[ids[0]][8:90] + (f" (+{len(ids)-1})" if len(ids) > 1 else "")
    print(f"{kind:5s} {d:9.2f} us {by/ d / 1e3 if by else 0:8.1f} GB/s {by/2**20:8.2f} MiB  {desc}")
print(tot)
