#!/usr/bin/env python3
"""Match a rocprofv3 kernel trace of `rank_sim.py C4 8` (last execute) to the plan's op list and
print per-op duration and algorithmic GB/s (sweep / apply / gemm)."""
import csv, re, sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch
import tneq_qc_amd  # noqa
from tneq_qc_amd.circuits import config_task
from tneq_qc_amd.expression import HipContractExpression

t = config_task("C4")
e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
p = e.plan(torch.complex64)
ops = p.describe().splitlines()
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"] and "splitk" not in r["Kernel_Name"]]
rows = rows[-len(ops):]
tot = {}
for op, r in zip(ops, rows):
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    m = re.search(r"tin=(\d+) tout=(\d+) cols=(\d+)", op)
    gbs = ""
    if m:
        tin, tout, cols = map(int, m.groups())
        gbs = f"{(tin + tout) * cols * 8 / d / 1e3:8.1f} GB/s"
    kind = op.split()[3] if op.startswith("[") else "?"
    tot[kind] = tot.get(kind, 0) + d
    print(f"{d:9.2f} us {gbs:>14}  {op[:110]}  | {r['Kernel_Name'][:40]}")
print(tot)
