#!/usr/bin/env python3
"""HBM roofline of the permute kernel (north_star: "rocprof HBM GB/s on the permute").

For binary-leg tensors of rank 20..28 (2^20..2^28 elements; complex64 and complex128) and seeded
random permutations, runs tq_permute through a one-op plan (the same kernel the contraction
plans launch before a GEMM, reference sites: the tensordot transposes under
einsum_strategy.py:639-643 and permute(...).contiguous() at distributed_engine.py:1330,1635),
times every launch with HIP events, checks the result bit-exactly on the smaller sizes, and
prints one JSON line per (dtype, rank, permutation): algorithmic bytes 2 * numel * sizeof,
GB/s and the fraction of the 8 TB/s HBM3E peak.

    python scripts/permute_bench.py [--ranks 20,22,24,26,28] [--dtypes c64,c128] [--perms 3] [--reps 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tneq_qc_amd import _lib  # noqa: E402
from tneq_qc_amd.einsum import get_symbol  # noqa: E402
from tneq_qc_amd.expression import HipContractExpression  # noqa: E402

PEAK = 8000.0
DT = {"c64": torch.complex64, "c128": torch.complex128, "f32": torch.float32, "f64": torch.float64}


def run(rank, dtype, perm, reps, check):
    s = "".join(get_symbol(i) for i in range(rank))
    e = HipContractExpression(s + "->" + "".join(s[i] for i in perm), (2,) * rank)
    x = torch.randn((2,) * rank, dtype=DT[dtype], device="cuda")
    y = torch.empty_like(x)
    e(x, out=y)
    plan = e.plan(DT[dtype])
    plan.profile(_lib.TQ_OP_PERMUTE)
    for _ in range(reps):
        e(x, out=y)
    torch.cuda.synchronize()
    r = plan.profile_read(_lib.TQ_OP_PERMUTE)
    plan.profile(None)
    ok = None
    if check:
        # on the host (torch's device permute stops at 16 dims)
        ok = bool(np.array_equal(y.cpu().numpy(), np.transpose(x.cpu().numpy(), [int(v) for v in perm])))
    gbs = r["bytes"] / (r["ms"] / 1e3) / 1e9
    return {"dtype": dtype, "rank": rank, "numel": 2 ** rank, "perm": [int(v) for v in perm],
            "avg_launch_ms": r["ms"] / r["launches"], "launches": r["launches"],
            "bytes_per_launch": r["bytes"] / r["launches"], "GBps": gbs, "frac": gbs / PEAK,
            "bit_exact": ok, "plan": plan.describe().splitlines()[0]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="20,22,24,26,28")
    ap.add_argument("--dtypes", default="c64,c128")
    ap.add_argument("--perms", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    rng = np.random.default_rng(2026)
    for dtype in a.dtypes.split(","):
        for rank in [int(v) for v in a.ranks.split(",")]:
            for _ in range(a.perms):
                p = rng.permutation(rank)
                print(json.dumps(run(rank, dtype, p, a.reps, check=rank <= 26)), flush=True)
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
