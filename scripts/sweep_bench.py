#!/usr/bin/env python3
"""Micro-benchmark of one fused sweep op: a 2^n-element running tensor (binary legs) absorbing a
chain of (2,2,2,2) gates on chosen legs.  Prints the plan's op and the achieved algorithmic
GB/s ((numel(X) + numel(Y)) * 8 B per launch) for a few leg placements."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import tneq_qc_amd  # noqa
from tneq_qc_amd.expression import HipContractExpression

SYM = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"


def case(n, pairs, reps=20, dev="cuda"):
    legs = list(SYM[:n])
    terms = ["".join(legs)]
    nxt = n
    cur = legs[:]
    for (p, q) in pairs:
        a, b = cur[p], cur[q]
        na, nb = SYM[nxt], SYM[nxt + 1]
        nxt += 2
        terms.append(a + b + na + nb)
        cur[p], cur[q] = na, nb
    eq = ",".join(terms) + "->" + "".join(cur)
    shapes = [tuple([2] * len(t)) for t in terms]
    path = [(0, 1)] + [(len(terms) + i, i + 2) for i in range(len(terms) - 2)]
    e = HipContractExpression(eq, *shapes, optimize=path)
    plan = e.plan(torch.complex64)
    rng = np.random.default_rng(0)
    ts = [torch.randn(s, dtype=torch.complex64, device=dev) for s in shapes]
    out = torch.empty(e.out_shape, dtype=torch.complex64, device=dev)
    for _ in range(3):
        e(*ts, out=out)
    torch.cuda.synchronize()
    plan.profile(-1)
    for _ in range(reps):
        e(*ts, out=out)
    torch.cuda.synchronize()
    r = plan.profile_read(-1)
    plan.profile(None)
    dt = r["ms"] / reps * 1e-3
    gbs = r["bytes"] / reps / dt / 1e9
    ops = [l for l in plan.describe().splitlines() if not l.startswith("#")]
    print(f"n={n} pairs={pairs}: {dt*1e6:8.1f} us GPU ({r['launches']//reps} launches)  {gbs:7.1f} GB/s", flush=True)
    for o in ops:
        print("    ", o[:110])


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    case(n, [(n - 1, n - 2)])                                 # one gate, innermost legs
    case(n, [(0, 1)])                                         # one gate, outermost legs
    case(n, [(n - 1, n - 2), (n - 3, n - 4)])                 # innermost legs
    case(n, [(n - 1, n - 2), (n - 3, n - 4), (n - 2, n - 3), (n - 1, n - 4)])
    case(n, [(0, 1), (2, 3)])                                 # outermost legs
    case(n, [(0, 1), (2, 3), (1, 2), (0, 3)])
    case(n, [(8, 9), (10, 11), (9, 10), (8, 11)])             # middle legs
    case(n, [(n - 1, 0), (n - 2, 1)])                         # mixed
