#!/usr/bin/env python3
"""Latency of one sweep launch on small tensors (the hoisted chains of C4 work on 2^19-2^20
elements): a 2^n binary tensor absorbing a chain of 8 (2,2,2,2) gates on its innermost legs.
Prints GPU microseconds per launch (plan profiling events) for n in argv."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tneq_qc_amd  # noqa
from tneq_qc_amd.expression import HipContractExpression

SYM = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"


def case(n, pairs, reps=50):
    legs = list(SYM[:n]); terms = ["".join(legs)]; nxt = n; cur = legs[:]
    for (p, q) in pairs:
        a, b = cur[p], cur[q]; na, nb = SYM[nxt], SYM[nxt + 1]; nxt += 2
        terms.append(a + b + na + nb); cur[p], cur[q] = na, nb
    eq = ",".join(terms) + "->" + "".join(cur)
    shapes = [tuple([2] * len(t)) for t in terms]
    path = [(0, 1)] + [(len(terms) + i, i + 2) for i in range(len(terms) - 2)]
    e = HipContractExpression(eq, *shapes, optimize=path)
    plan = e.plan(torch.complex64)
    ts = [torch.randn(s, dtype=torch.complex64, device="cuda") for s in shapes]
    out = torch.empty(e.out_shape, dtype=torch.complex64, device="cuda")
    for _ in range(3):
        e(*ts, out=out)
    torch.cuda.synchronize()
    plan.profile(-1)
    for _ in range(reps):
        e(*ts, out=out)
    torch.cuda.synchronize()
    r = plan.profile_read(-1)
    rs = plan.profile_read(4)   # TQ_OP_SWEEP (sweep2 launches are profiled as SWEEP)
    plan.profile(None)
    ops = [l for l in plan.describe().splitlines() if "SWEEP2" in l]
    us = rs['ms'] / reps * 1e3
    gbs = rs['bytes'] / reps / (us * 1e-6) / 1e9 if us else 0
    print(f"n={n}: {r['ms'] / reps * 1e3:7.1f} us/execute ({r['launches'] // reps} launches), sweep {us:7.1f} us "
          f"{gbs:6.0f} GB/s; {ops[0][:100] if ops else ''}", flush=True)


for n in [int(a) for a in sys.argv[1:]] or [19, 20, 22]:
    k = n - 8
    case(n, [(k + 7, k + 6), (k + 5, k + 4), (k + 3, k + 2), (k + 1, k), (k + 6, k + 5), (k + 4, k + 3), (k + 2, k + 1), (k + 7, k)])
