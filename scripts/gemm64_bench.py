#!/usr/bin/env python3
"""MFMA GEMMs through the C ABI vs torch.matmul (rocBLAS / hipBLASLt) on the same shapes; prints
TF/s and the fraction of the FP64 (78.6 TF/s) / FP32 (157.3 TF/s) MFMA peak ("executed" counts
the real MFMA flops: 6 MNK for the Gauss-3M complex kernels).  layout "mk": A is M x K (the
register-staged generic kernel); layout "kouter": A is K x M, B is K x N (the LDS-DMA fast
kernels: v_mfma_f64_16x16x4_f64 for f64 / complex128, v_mfma_f32_32x32x2_f32 for complex64).
    python scripts/gemm64_bench.py [f64 c128 c64 ...] [--layout mk|kouter|both]"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tneq_qc_amd.ops as ops

dev = torch.device("cuda:0")
PEAK = {torch.float64: 78.6, torch.complex128: 78.6, torch.float32: 157.3, torch.complex64: 157.3}
shapes = [(4096, 4096, 4096), (2048, 2048, 8192), (1024, 1024, 16384), (8192, 8192, 1024)]
args = [x for x in sys.argv[1:] if not x.startswith("--layout")]
lay = next((x.split("=")[1] for x in sys.argv[1:] if x.startswith("--layout=")), "both")
only = args or ["f64", "c128"]
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


def threem(dt):
    return dt.is_complex and os.environ.get("TQ_GEMM_3M", "1") != "0"


for name in only:
    dt = dts[name]
    for layout in (["mk", "kouter"] if lay == "both" else [lay]):
        for (M, N, K) in shapes:
            b = torch.randn(K, N, dtype=dt, device=dev)
            c = torch.empty(1, M, N, dtype=dt, device=dev)
            if layout == "mk":
                a = torch.randn(M, K, dtype=dt, device=dev)     # A M x K (K contiguous)
                fn = lambda: ops.gemm(a, b, False, False, out=c)
                ref = lambda: torch.matmul(a, b)
            else:
                a = torch.randn(K, M, dtype=dt, device=dev)     # A K x M (M contiguous)
                fn = lambda: ops.gemm(a, b, True, False, out=c)
                ref = lambda: torch.matmul(a.t(), b)
            fl = (8.0 if dt.is_complex else 2.0) * M * N * K
            fl_x = fl * (0.75 if (layout == "kouter" and threem(dt)) else 1.0)
            ms = t_ms(fn)
            ms_t = t_ms(ref)
            r0 = ref()
            err = ((c[0] - r0).abs().max() / r0.abs().max()).item()
            r = {"dtype": name, "layout": layout, "MNK": [M, N, K], "ms": ms, "tflops": fl / ms / 1e9,
                 "executed_tflops": fl_x / ms / 1e9, "frac_executed": fl_x / ms / 1e9 / PEAK[dt],
                 "torch_ms": ms_t, "torch_tflops": fl / ms_t / 1e9, "rel_err_vs_torch": err}
            print(json.dumps(r), flush=True)
            del a, b, c, r0
            torch.cuda.empty_cache()
