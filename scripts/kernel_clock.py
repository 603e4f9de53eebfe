#!/usr/bin/env python3
"""In-kernel clock of the benchmarked kernels, replacing the PMC estimate
GRBM_GUI_ACTIVE / 8 / duration (unphysical for short dispatches: 2.8-10.8 GHz in r05).  Needs the
-DTQ_KCLOCK build (csrc: make BUILD=../lib/obj_kclock OUT=../lib/libtneqhip_kclock.so
EXTRA=-DTQ_KCLOCK): workgroup 0 of every launch stamps s_memtime / s_memrealtime at its start and
end (tq_kclock.h); clock = d(memtime) / d(memrealtime) x 100 MHz.  Runs the C4 headline regime
(BlockPipeline, 4 blocks in flight, >= 2 s of back-to-back blocks) for sweep2 and the boundary
GEMM, then C4g for the planes GEMM.  One JSON object on stdout.
    TNEQHIP_LIB=<kclock build> python scripts/kernel_clock.py > profiles/kclock_r06.json"""
import ctypes, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tneq_qc_amd import _lib
from tneq_qc_amd.circuits import config_task
from tneq_qc_amd.expression import HipContractExpression
from tneq_qc_amd.sampling import BlockPipeline

L = _lib.lib()
f = L.tq_debug_kernel_clock
f.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
f.restype = ctypes.c_int
N = 4096
buf = (ctypes.c_ulonglong * (4 * N))()
NAMES = {0: "sweep2_kernel", 1: "gemm_planes_kernel", 2: "gemm_c64_kouter_split_kernel"}


def drain(which):
    n = f(which, buf, N)
    if n <= 0:
        return None
    a = np.frombuffer(buf, dtype=np.uint64, count=4 * n).reshape(n, 4).astype(np.float64)
    dmt, drt = a[:, 2] - a[:, 0], a[:, 3] - a[:, 1]
    ok = drt >= 100   # >= 1 us of workgroup 0's lifetime (100 MHz ticks): quantisation < 1 %
    if not ok.any():
        return {"records": int(n), "used": 0}
    ghz = dmt[ok] / drt[ok] / 10.0
    return {"records": int(n), "used": int(ok.sum()), "clock_GHz_median": float(np.median(ghz)),
            "clock_GHz_p10": float(np.percentile(ghz, 10)), "clock_GHz_p90": float(np.percentile(ghz, 90)),
            "wg0_lifetime_us_median": float(np.median(drt[ok]) / 100.0)}


dev = torch.device("cuda:0")
out = {"method": "workgroup 0 of every launch: (s_memtime end - start) / (s_memrealtime end - start) x 100 MHz "
                 "(tq_kclock.h, -DTQ_KCLOCK build); launches whose workgroup 0 lived >= 1 us",
       "peak_clock_GHz": 2.4}
pipe = BlockPipeline(config_task("C4"), list(range(64)), inflight=4, device=dev)
t0 = time.time()
while time.time() - t0 < 2.0:
    for _ in range(16):
        pipe.step()
    pipe.synchronize()
for w in (0, 2):
    drain(w)
for _ in range(64):
    pipe.step()
pipe.synchronize()
out["C4_headline_regime"] = {NAMES[w]: drain(w) for w in (0, 2)}
del pipe
t = config_task("C4g")
e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in t.operands]
o = torch.empty(e.out_shape, dtype=torch.complex64, device=dev)
for _ in range(3):
    e(*ops, out=o)
torch.cuda.synchronize()
drain(1)
for _ in range(4):
    e(*ops, out=o)
torch.cuda.synchronize()
out["C4g"] = {NAMES[1]: drain(1)}
print(json.dumps(out, indent=1))
