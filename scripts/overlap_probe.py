#!/usr/bin/env python3
"""Probe: does HBM-bound work hide under the power-limited boundary GEMM?

The C4 step runs two 4-lane batches, each = per-slice sweeps (HBM-bound, ~1.2 ms) then the
batched f16-split GEMM (~5.5 ms, MFMA busy ~67 %).  This times the lane-batched GEMM of the bench
shape (4 x 1024 x 1024 x 65536) alone, a stream of HBM copies alone (~2.4 GiB moved, like one
batch's sweeps), both one after the other, and both concurrently on two streams.
    python scripts/overlap_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tneq_qc_amd.ops as ops  # noqa: E402

dev = torch.device("cuda:0")
B, M, N, K = 4, 1024, 1024, 65536
g = torch.Generator(device=dev).manual_seed(1)
a = torch.randn(B, K, M, dtype=torch.complex64, device=dev, generator=g)
b = torch.randn(B, K, N, dtype=torch.complex64, device=dev, generator=g)
c = torch.empty(B, M, N, dtype=torch.complex64, device=dev)
x = torch.randn(2 ** 27, dtype=torch.complex64, device=dev)   # 1 GiB
y = torch.empty_like(x)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def gemm():
    ops.gemm(a, b, True, False, out=c)


def copies():
    for _ in range(1):
        y.copy_(x)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def conc():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        gemm()
    with torch.cuda.stream(s2):
        copies()
    cur.wait_stream(s1)
    cur.wait_stream(s2)


res = {"gemm_ms": timed(gemm), "copies_ms": timed(copies),
       "sequential_ms": timed(lambda: (gemm(), copies())), "concurrent_ms": timed(conc)}
res["copy_GBps"] = 2 * x.numel() * 8 / (res["copies_ms"] / 1e3) / 1e9
res["hidden_frac"] = (res["sequential_ms"] - res["concurrent_ms"]) / res["copies_ms"]
print(json.dumps(res), flush=True)
