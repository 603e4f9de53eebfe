#!/usr/bin/env python3
"""the measured complex64 error of every benchmarked production launch (the
whole job as bench.py runs it: SlicedContraction over all slices, captured hipGraph replayed)
against the exact complex128 sum over all slices (oracle.contract_ref.contract_sliced), next to
the error of the oracle's own numpy pairwise executor run in complex64 on the same job (what a
plain fp32 CPU contraction of the same path achieves).  Normwise = max|err| / max|amp|;
componentwise = max |err| / |amp| over |amp| >= 1e-2 max|amp|.  One JSON line."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import tneq_qc_amd  # noqa: F401
from tneq_qc_amd.circuits import config_task
from tneq_qc_amd.distributed import SlicedContraction
from tneq_qc_amd.expression import HipContractExpression
from oracle.contract_ref import contract_sliced


def errs(got, ref):
    amax = np.abs(ref).max()
    err = np.abs(got - ref)
    big = np.abs(ref) >= 1e-2 * amax
    return {"normwise": float(err.max() / amax), "componentwise_ge_1e-2max": float((err[big] / np.abs(ref[big])).max()),
            "rms_rel": float(np.sqrt((err ** 2).mean()) / np.sqrt((np.abs(ref) ** 2).mean()))}


dev = torch.device("cuda:0")
out = {"definition": __doc__.split("\n\n")[0], "configs": {}}
exact = {}
for cfg in sys.argv[1:] or ["C4", "C4g", "C3", "C3d", "C4x4"]:
    t = config_task(cfg)
    base = {"C3d": "C3", "C4g": "C4"}.get(cfg, cfg)
    t0 = time.time()
    if base not in exact:
        tb = config_task(base)
        exact[base] = contract_sliced(tb.eq, tb.operands, tb.sliced, tb.path)
    ref = exact[base]
    e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
    ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in t.operands]
    job = SlicedContraction(e)
    o = torch.empty(e.out_shape, dtype=torch.complex64, device=dev)
    for _ in range(3):
        job(*ops, out=o)
    got = o.cpu().numpy()
    r = {"gpu_c64": errs(got, ref)}
    if cfg == base:   # (C4g's big-GEMM path is hours of numpy)
        c64 = contract_sliced(t.eq, [x.astype(np.complex64) for x in t.operands], t.sliced, t.path, exact=False)
        r["numpy_c64_same_path"] = errs(np.asarray(c64), ref)
    r["seconds"] = round(time.time() - t0, 1)
    out["configs"][cfg] = r
    print(cfg, json.dumps(r), file=sys.stderr, flush=True)
print(json.dumps(out))
