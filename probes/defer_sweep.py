"""Time the whole-job contraction (bench.py's launch: SlicedContraction at world 1, captured graph
replayed) of a config's network over several deferred-tail splits (einsum.partition_path
defer=(left, right)), and check every split gives the same amplitudes.

    python probes/defer_sweep.py C3 [ns=K] 0,0 4,4 10,8 ...     (ns: sliced cut legs, default the config's)
"""
import sys
import time

import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from tneq_qc_amd import einsum as E
from tneq_qc_amd.circuits import BrickWall, amplitude_task
from tneq_qc_amd.distributed import SlicedContraction
from tneq_qc_amd.expression import HipContractExpression

ARGS = {"C3": (BrickWall(40, 16, 0), list(range(12, 28)), 20, 6),
        "C4": (BrickWall(53, 20, 0), list(range(17, 37)), 27, 3)}


def main():
    cfg = sys.argv[1]
    circ, opn, cut, ns = ARGS[cfg]
    dev = torch.device("cuda:0")
    ref = None
    specs = sys.argv[2:]
    if specs and specs[0].startswith("ns="):
        ns = int(specs[0][3:])
        specs = specs[1:]
    for spec in specs:
        d = tuple(int(x) for x in spec.split(","))
        t = amplitude_task(circ, opn, cut=cut, n_slice=ns, defer=d)
        net = E.parse_equation(t.eq, t.shapes)
        fl = E.path_info(net, t.path, [net.symbols.index(x) for x in t.sliced]).flops
        e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
        ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in t.operands]
        job = SlicedContraction(e)
        out = torch.empty(e.out_shape, dtype=torch.complex64, device=dev)
        for _ in range(3):
            job(*ops, out=out)
        torch.cuda.synchronize()
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            job(*ops, out=out)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / n * 1e3
        got = out.cpu().numpy()
        if ref is None:
            ref = got
        err = np.abs(got - ref).max() / np.abs(ref).max()
        p = e.plan(torch.complex64)
        print(f"{cfg} defer={d} flops={fl:.3g} slices={e.n_slices} lanes={p.query('lanes')} "
              f"ms={ms:.3f} err_vs_first={err:.2e}", flush=True)
        del e, job, ops, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
