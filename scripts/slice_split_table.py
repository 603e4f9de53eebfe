#!/usr/bin/env python3
"""can the slice (RCCL) path of the DEFERRED C4 network divide its hoisted
sweeps across ranks?  For each candidate slicing, the planner's roofline model (einsum.path_info:
one launch + max(bytes / 5 TB/s, MACs / 110 TF/s) per pairwise step) of a whole 1-GPU execute and
of ONE rank of an 8-GPU split (hoisted part replicated, slices dealt round-robin).  Candidates:
the config's cut-leg slicing (choose_slices over the cut legs), a greedy over EVERY contracted
mode minimising the rank-8 time (+0.2 x the 1-GPU time), and C4g (the big-GEMM path) for
comparison.  Host only (no GPU).  Usage: python scripts/slice_split_table.py > profiles/slice_split_r06.json"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tneq_qc_amd.circuits import config_task  # noqa: E402
from tneq_qc_amd.einsum import path_info  # noqa: E402


def row(name, net, path, sl):
    i = path_info(net, path, sl)
    r8 = i.est_ranks(8)
    return {"slicing": name, "sliced_modes": [net.symbols[m] for m in sl], "n_slices": i.n_slices,
            "est_1gpu_ms": round(i.est_seconds * 1e3, 3), "est_rank8_ms": round(r8 * 1e3, 3),
            "proj_speedup_N8": round(i.est_seconds / r8, 2), "hoisted_ms": round(i.t_once * 1e3, 3),
            "per_slice_ms": round(i.t_slice * 1e3, 4), "complex_macs": i.flops}


out = {"model": "einsum.path_info roofline (2 us launch + max(bytes/5 TB/s, MACs/110 TF/s) per pairwise step)",
       "rows": []}
for cfg in ("C4", "C4g"):
    t = config_task(cfg)
    net = t.network()
    sym = {s: i for i, s in enumerate(net.symbols)}
    out["rows"].append(dict(row("cut legs (config)", net, t.path, [sym[s] for s in t.sliced]), config=cfg))
    if cfg != "C4":
        continue
    out["rows"].append(dict(row("none", net, t.path, []), config=cfg))
    t0 = time.time()
    cands = [m for m in net.extents if m not in set(net.out)]
    chosen = []
    for _ in range(len(t.sliced)):
        best = None
        for m in cands:
            if m in chosen:
                continue
            i = path_info(net, t.path, chosen + [m])
            key = (i.est_ranks(8) + 0.2 * i.est_seconds, m)
            if best is None or key < best[0]:
                best = (key, m)
        chosen.append(best[1])
        out["rows"].append(dict(row(f"greedy over all {len(cands)} contracted modes ({len(chosen)})", net, t.path,
                                    list(chosen)), config=cfg))
    out["greedy_seconds"] = round(time.time() - t0, 1)
print(json.dumps(out, indent=1))
