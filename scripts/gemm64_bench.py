#!/usr/bin/env python3
"""Generic MFMA GEMM (f64 / complex128 v_mfma_f64_16x16x4_f64, f32 / complex64 non-K-outer)
through the C ABI vs torch.matmul (rocBLAS / hipBLASLt) on the same shapes; prints TF/s and the
fraction of the FP64 (78.6 TF/s) / FP32 (157.3 TF/s) MFMA peak."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tneq_qc_amd.ops as ops

dev = torch.device("cuda:0")
PEAK = {torch.float64: 78.6, torch.complex128: 78.6, torch.float32: 157.3, torch.complex64: 157.3}
shapes = [(4096, 4096, 4096), (2048, 2048, 8192), (1024, 1024, 16384), (8192, 8192, 1024)]
only = sys.argv[1:] if len(sys.argv) > 1 else ["f64", "c128"]
dts = {"f64": torch.float64, "c128": torch.complex128, "f32": torch.float32, "c64": torch.complex64}


def t_ms(fn, reps=5):
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


for name in only:
    dt = dts[name]
    for (M, N, K) in shapes:
        a = torch.randn(M, K, dtype=dt, device=dev)     # A M x K (K contiguous), B K x N
        b = torch.randn(K, N, dtype=dt, device=dev)
        c = torch.empty(1, M, N, dtype=dt, device=dev)
        fl = (8.0 if dt.is_complex else 2.0) * M * N * K
        ms = t_ms(lambda: ops.gemm(a, b, False, False, out=c))
        ms_t = t_ms(lambda: torch.matmul(a, b))
        err = ((c[0] - torch.matmul(a, b)).abs().max() / torch.matmul(a, b).abs().max()).item()
        r = {"dtype": name, "MNK": [M, N, K], "ms": ms, "tflops": fl / ms / 1e9,
             "frac": fl / ms / 1e9 / PEAK[dt], "torch_ms": ms_t, "torch_tflops": fl / ms_t / 1e9,
             "rel_err_vs_torch": err}
        print(json.dumps(r), flush=True)
        del a, b, c
        torch.cuda.empty_cache()
