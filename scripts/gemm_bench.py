#!/usr/bin/env python3
"""Time the boundary-GEMM shape (complex64, A K x M, B K x N) through the C ABI; run once with
TQ_GEMM_FAST=0 and once with the default to A/B the generic and the LDS-DMA kernels."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tneq_qc_amd.ops as ops

dev = torch.device("cuda:0")
res = {"fast": os.environ.get("TQ_GEMM_FAST", "1")}
for (M, N, K) in [(1024, 1024, 65536), (1024, 1024, 131072), (2048, 2048, 16384), (4096, 4096, 4096)]:
    a = torch.randn(K, M, dtype=torch.complex64, device=dev)
    b = torch.randn(K, N, dtype=torch.complex64, device=dev)
    c = torch.empty(1, M, N, dtype=torch.complex64, device=dev)
    for _ in range(2):
        ops.gemm(a, b, True, False, out=c)
    torch.cuda.synchronize()
    reps = 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.gemm(a, b, True, False, out=c)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    res[f"{M}x{N}x{K}"] = {"ms": ms, "tflops": 8.0 * M * N * K / ms / 1e9}
    del a, b, c
print(json.dumps(res))
