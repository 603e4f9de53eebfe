#!/usr/bin/env python3
"""Accuracy of the benchmarked C4 path on one slice, against the oracle (exact complex128 numpy).

Runs slice `sid` of the C4 bench configuration (53q d20, cut 27, 3 sliced cut legs) through the
native plan in complex64 (fast GEMM: Gauss 3M by default, 4M with TQ_GEMM_3M=0) and complex128,
and reports normwise error (max |err| / max |amp|) and componentwise error (|err| / |amp|) over
amplitude-magnitude bands.  Writes one JSON line to stdout (and `--out` if given).

    python scripts/accuracy_c4.py [--slice 0] [--config C4] [--out profiles/accuracy_r02.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tneq_qc_amd  # noqa: F401,E402
from tneq_qc_amd import _lib  # noqa: E402
from tneq_qc_amd.circuits import config_task  # noqa: E402
from tneq_qc_amd.expression import HipContractExpression  # noqa: E402
from oracle.contract_ref import contract as ref_contract, sliced_operands  # noqa: E402


def stats(got, ref):
    amax = np.abs(ref).max()
    err = np.abs(got - ref)
    out = {"normwise": float(err.max() / amax)}
    a = np.abs(ref)
    for lo in (1e-1, 1e-2, 1e-3, 1e-4):
        m = a >= lo * amax
        out[f"componentwise_max_ge_{lo:g}max"] = float((err[m] / a[m]).max()) if m.any() else None
        out[f"n_ge_{lo:g}max"] = int(m.sum())
    out["componentwise_median"] = float(np.median(err / np.maximum(a, 1e-300)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--slice", type=int, default=0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    t = config_task(a.config)
    e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
    eq, sops = sliced_operands(t.eq, t.operands, t.sliced, a.slice)
    ref = ref_contract(eq, *sops, path=t.path)
    res = {"config": a.config, "slice": a.slice,
           "gemm_3m": int(_lib.lib().tq_library_query(b"gemm_3m")), "n_amplitudes": int(ref.size)}
    for dt in (torch.complex64, torch.complex128):
        ops = [torch.from_numpy(o).to("cuda", dt) for o in t.operands]
        got = e(*ops, slice_range=(a.slice, a.slice + 1, 1)).cpu().numpy()
        res[str(dt).replace("torch.", "")] = stats(got, ref)
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "a") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
