#!/usr/bin/env python3
"""complex64 K-outer GEMM (A K x M, B K x N; the boundary GEMM of the C4 slices) through the C ABI:
time, TF/s (algorithmic 8 MNK and executed MFMA flops) and error against a complex128 reference.
Run once per kernel: default (f16 2-term split of the scaled operands) / TQ_GEMM_F16=0 (bf16
3-term split) / TQ_GEMM_BF16=0 (f32 MFMA).
    python scripts/gemm_c64_bench.py [--reps N]"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tneq_qc_amd.ops as ops
from tneq_qc_amd import _lib

dev = torch.device("cuda:0")
reps = int(next((a.split("=")[1] for a in sys.argv[1:] if a.startswith("--reps=")), 10))
L = _lib.lib()
bf16 = L.tq_library_query(b"gemm_bf16") == 1
f16 = bf16 and L.tq_library_query(b"gemm_f16") == 1
g3m = L.tq_library_query(b"gemm_3m") == 1
shapes = [(1024, 1024, 65536), (1024, 1024, 8192), (2048, 2048, 16384), (4096, 4096, 4096)]
if "--bench-shape" in sys.argv:
    shapes = shapes[:1]


def t_ms(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for (M, N, K) in shapes:
    g = torch.Generator(device=dev).manual_seed(1)
    a = torch.randn(K, M, dtype=torch.complex64, device=dev, generator=g)
    b = torch.randn(K, N, dtype=torch.complex64, device=dev, generator=g)
    c = torch.empty(1, M, N, dtype=torch.complex64, device=dev)
    fn = lambda: ops.gemm(a, b, True, False, out=c)
    ms = t_ms(fn)
    ref = torch.matmul(a.t().to(torch.complex128), b.to(torch.complex128))
    err = ((c[0].to(torch.complex128) - ref).abs().max() / ref.abs().max()).item()
    fl = 8.0 * M * N * K
    if f16:
        fl_x, peak, unit = 12 * 2.0 * M * N * K, 2500.0, "f16 MFMA"
    elif bf16:
        fl_x, peak, unit = 24 * 2.0 * M * N * K, 2500.0, "bf16 MFMA"
    else:
        fl_x, peak, unit = (6.0 if g3m else 8.0) * M * N * K, 157.3, "f32 MFMA"
    print(json.dumps({"kernel": "f16x2-split" if f16 else "bf16x3-split" if bf16 else ("f32-3M" if g3m else "f32-4M"), "MNK": [M, N, K],
                      "ms": ms, "algorithmic_tflops": fl / ms / 1e9, "executed_tflops": fl_x / ms / 1e9,
                      "peak": peak, "frac_executed": fl_x / ms / 1e9 / peak, "mfma": unit,
                      "rel_err_vs_c128": err}), flush=True)
    del a, b, c, ref
    torch.cuda.empty_cache()
