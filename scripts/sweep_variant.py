#!/usr/bin/env python3
"""Development aid: runs whole C4 executes (all slices) a few times, for a rocprofv3 kernel trace
of the sweep2 launches under a build / environment variant (scripts/r02_s46.sh)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tneq_qc_amd.circuits import config_task
from tneq_qc_amd.expression import HipContractExpression

task = config_task(sys.argv[1] if len(sys.argv) > 1 else "C4")
expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
dev = torch.device("cuda:0")
ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in task.operands]
out = torch.empty(expr.out_shape, dtype=torch.complex64, device=dev)
for _ in range(4):
    expr(*ops, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    expr(*ops, out=out)
e1.record()
torch.cuda.synchronize()
print(f"ms_per_execute {e0.elapsed_time(e1) / 10:.3f} max|amp| {float(out.abs().max()):.6e}")
