#!/usr/bin/env python3
"""Phase timing of every sweep2 op of one C4 execute (development aid).  Needs libtneqhip.so
built with -DTQ_S2_TIMING (csrc: make BUILD=../lib/obj_timing OUT=../lib/libtneqhip_timing.so EXTRA=-DTQ_S2_TIMING): workgroup 0 of each op stamps the wall
clock (100 MHz) at: start, descriptor staged, tables built, first chunk in LDS, first chunk's
gates done, first chunk stored, end.  Prints per-op phase durations in us.
    TNEQHIP_LIB=<timing build> python scripts/sweep_timing.py [C4|C3|C2] [slices] [--group G]"""
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
NREC, W = 2048, 48
buf = (ctypes.c_ulonglong * (NREC * W))()
import argparse
ap = argparse.ArgumentParser()
ap.add_argument("config", nargs="?", default="C4")
ap.add_argument("slices", nargs="?", type=int, default=1)
ap.add_argument("--group", type=int, default=1, help="time one lockstep group of G blocks (BlockPipeline)")
args = ap.parse_args()
task = config_task(args.config)
dev = torch.device("cuda:0")
if args.group > 1:
    from tneq_qc_amd.sampling import BlockPipeline
    pipe = BlockPipeline(task, list(range(args.group)), inflight=1, group=args.group, device=dev)

    def run():
        for _ in range(args.group):
            pipe.step()
        pipe.synchronize()
else:
    expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
    ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in task.operands]
    out = torch.empty(expr.out_shape, dtype=torch.complex64, device=dev)
    SR = (0, args.slices, 1)   # slices of the timed execute

    def run():
        expr(*ops, out=out, slice_range=SR)
        torch.cuda.synchronize()
for _ in range(3):
    run()
f(buf, NREC)  # drain
run()
n = f(buf, NREC)
a = np.frombuffer(buf, dtype=np.uint64, count=n * W).reshape(n, W).astype(np.int64)
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
# tables phase split (stamps 41-43, thread 0 of workgroup 0): lane offsets + first chunk's loads
# issued / coefficients staged / tables staged / barrier
sub = np.zeros(4)
for r in a:
    t1, t41, t42, t43, t2 = r[1], r[41], r[42], r[43], r[2]
    if min(t41, t42, t43) > 0:
        sub += np.array([t41 - t1, t42 - t41, t43 - t42, t2 - t43]) / 100.0
print("tables phase split (sum, us):", json.dumps(dict(zip(["lane_offs+chunk0_issue", "coeffs", "tables", "barrier"], np.round(sub, 1).tolist()))))
# the first part in detail (stamps 44-47: next descriptor issued, lane offsets, chunk bases,
# cooperative wait; 41: first chunk's loads issued)
sub = np.zeros(5)
for r in a:
    t = [r[1], r[44], r[45], r[46], r[47], r[41]]
    if min(t) > 0:
        sub += np.diff(np.array(t)) / 100.0
print("lane_offs+chunk0_issue split (sum, us):", json.dumps(dict(zip(["next_desc_issue", "lane_offsets", "chunk_bases", "coop_wait", "chunk0_issue"], np.round(sub, 1).tolist()))))
# per-pass clocks of the first chunk (shader clock), grouped by pass kind
kinds = {}
for r in a:
    prev = 0
    for p in range(16):
        t = int(r[9 + p])
        if t == 0:
            break
        k = int(r[25 + p])
        key = (f"B{(k >> 16) & 0xff}x{k >> 24}" if (k >> 16) & 0xff else f"{(k >> 8) & 0xff}x{k & 0xff}")
        kinds.setdefault(key, []).append(t - prev)
        prev = t
print("per-pass clocks (first chunk, WG0): kind -> (count, median, mean)")
for k, v in sorted(kinds.items(), key=lambda kv: -len(kv[1])):
    print(f"  {k:8s} {len(v):4d} {int(np.median(v)):7d} {int(np.mean(v)):7d}")
