#!/usr/bin/env python3
"""Time the skinny contraction shapes of the C5 reverse tree (complex128) through ops.gemm, all four
transpositions; run once with TQ_GEMM_SKINNY=0 (tiled MFMA kernels + split-K) and once without.
    python scripts/skinny_bench.py"""
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tneq_qc_amd.ops as ops  # noqa: E402

dev = torch.device("cuda:0")
out = {"skinny": os.environ.get("TQ_GEMM_SKINNY", "1")}
for (M, N, K) in [(4, 4, 16384), (8, 2, 8192), (2, 8, 512), (4, 4, 1024), (4, 4, 64)]:
    for ta, tb in itertools.product((False, True), (False, True)):
        a = torch.randn((K, M) if ta else (M, K), dtype=torch.complex128, device=dev)
        b = torch.randn((N, K) if tb else (K, N), dtype=torch.complex128, device=dev)
        c = torch.empty(1, M, N, dtype=torch.complex128, device=dev)
        for _ in range(3):
            ops.gemm(a, b, ta, tb, out=c)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            ops.gemm(a, b, ta, tb, out=c)
        e1.record()
        torch.cuda.synchronize()
        out[f"{M}x{N}x{K} t{int(ta)}{int(tb)}"] = round(e0.elapsed_time(e1) / 50 * 1e3, 1)
print(json.dumps(out), flush=True)
