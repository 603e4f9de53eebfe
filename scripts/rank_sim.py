#!/usr/bin/env python3
"""Time what one rank of an N-GPU run executes (slices r, r+N, ...) on a single GPU, to project
the multi-GPU per-rank time from a 1-GPU box (no collective; the RCCL reduce of 8 MiB is ~0.1 ms)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tneq_qc_amd  # noqa
from tneq_qc_amd.circuits import config_task
from tneq_qc_amd.expression import HipContractExpression

cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
only = [int(sys.argv[2])] if len(sys.argv) > 2 else None   # e.g. 8: time only rank 0 of N=8
dev = torch.device("cuda:0")
task = config_task(cfg)
expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in task.operands]
out = torch.empty(expr.out_shape, dtype=torch.complex64, device=dev)
ns = expr.n_slices
res = {"config": cfg, "slices": ns}
for world in (only or (1, 2, 4, 8)):
    if world > ns:
        break
    rng = (0, ns, world)
    for _ in range(2):
        expr(*ops, out=out, slice_range=rng)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        expr(*ops, out=out, slice_range=rng)
    torch.cuda.synchronize()
    res[f"rank_ms_N{world}"] = (time.perf_counter() - t0) / reps * 1e3
for w in (2, 4, 8):
    if f"rank_ms_N{w}" in res and "rank_ms_N1" in res:
        res[f"proj_speedup_N{w}"] = res["rank_ms_N1"] / res[f"rank_ms_N{w}"]
print(json.dumps(res))
