#!/usr/bin/env python3
"""Phase timing of every sweep2 op of one C4 execute (development aid).  Needs libtneqhip.so
built with -DTQ_S2_TIMING (make EXTRA=-DTQ_S2_TIMING): workgroup 0 of each op stamps the wall
clock (100 MHz) at: start, descriptor staged, tables built, first chunk in LDS, first chunk's
gates done, first chunk stored, end.  Prints per-op phase durations in us."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tneq_qc_amd import _lib
from tneq_qc_amd.circuits import config_task
from tneq_qc_amd.expression import HipContractExpression

L = _lib.lib()
f = L.tq_debug_sweep2_timing
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
f.restype = ctypes.c_int
buf = (ctypes.c_ulonglong * (4096 * 9))()
task = config_task(sys.argv[1] if len(sys.argv) > 1 else "C4")
expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
dev = torch.device("cuda:0")
ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in task.operands]
out = torch.empty(expr.out_shape, dtype=torch.complex64, device=dev)
for _ in range(3):
    expr(*ops, out=out, slice_range=(0, 1, 1))
torch.cuda.synchronize()
f(buf, 4096)  # drain
expr(*ops, out=out, slice_range=(0, 1, 1))
torch.cuda.synchronize()
n = f(buf, 4096)
a = np.frombuffer(buf, dtype=np.uint64, count=n * 9).reshape(n, 9).astype(np.int64)
a = a[np.argsort(a[:, 0])]
t0 = a[0, 0]
names = ["desc", "tables", "chunk0_in", "gates0", "store0", "rest+drain"]
print(f"{n} op records (us from first start; phases: {names})")
tot = np.zeros(6)
for r in a:
    ph = np.diff(r[:7]) / 100.0  # 100 MHz
    tot += ph
    print(f"start {(r[0]-t0)/100:8.2f} end {(r[6]-t0)/100:8.2f} | " + " ".join(f"{x:6.2f}" for x in ph)
          + f" | wgs {int(r[7]) >> 32} chunks {int(r[7]) & 0xffffffff} | gate clk {r[8] / max(ph[3], 1e-3) / 1e3:6.0f} MHz")
print("sum per phase:", json.dumps(dict(zip(names, np.round(tot, 1).tolist()))))
