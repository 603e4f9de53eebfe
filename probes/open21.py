"""Cost of one contraction of TWO amplitude blocks at once (one more open qubit next to the open
range, 2^21 amplitudes) against one block (C4, 2^20), same cut / slicing, several deferred-tail
splits; one stream, whole executes timed.

    python probes/open21.py [lo] [hi] [l,r ...]      (open qubits lo..hi-1; default 16 37)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from tneq_qc_amd.circuits import BrickWall, amplitude_task
from tneq_qc_amd.expression import HipContractExpression


def run(task, dev, n=20):
    e = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
    ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in task.operands]
    out = torch.empty(e.out_shape, dtype=torch.complex64, device=dev)
    for _ in range(3):
        e(*ops, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        e(*ops, out=out)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    lo = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    hi = int(sys.argv[2]) if len(sys.argv) > 2 else 37
    specs = [tuple(int(x) for x in s.split(",")) for s in sys.argv[3:]] or [(20, 16)]
    dev = torch.device("cuda:0")
    circ = BrickWall(53, 20, 0)
    for d in specs:
        t = amplitude_task(circ, list(range(lo, hi)), cut=27, n_slice=3, defer=d)
        ms = run(t, dev)
        print(f"open {lo}..{hi - 1} ({hi - lo}) defer={d} slices={2 ** len(t.sliced)} ms={ms:.4f} "
              f"ms_per_2^20={ms / 2 ** (hi - lo - 20):.4f}", flush=True)


if __name__ == "__main__":
    main()
