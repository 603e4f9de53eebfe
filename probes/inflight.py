"""Throughput of M amplitude blocks in flight on one GPU: M plans (own arenas) of the C4 network,
step k on plan k % M's stream, each step one whole block.  Prints ms per block for M = 1..4.

    python probes/inflight.py [C4] [M ...]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from tneq_qc_amd.circuits import config_task, with_batch
from tneq_qc_amd.expression import HipContractExpression


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
    ms_list = [int(x) for x in sys.argv[2:]] or [1, 2, 3, 4]
    dev = torch.device("cuda:0")
    base = config_task(cfg)
    for m in ms_list:
        exprs, opss, outs, streams = [], [], [], []
        for i in range(m):
            t = with_batch(base, i)
            e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
            exprs.append(e)
            opss.append([torch.from_numpy(o).to(dev, torch.complex64) for o in t.operands])
            outs.append(torch.empty(e.out_shape, dtype=torch.complex64, device=dev))
            streams.append(torch.cuda.Stream(dev))

        def run(k):
            for s in range(k):
                i = s % m
                with torch.cuda.stream(streams[i]):
                    exprs[i](*opss[i], out=outs[i])

        run(3 * m)
        torch.cuda.synchronize()
        n = 40
        t0 = time.perf_counter()
        run(n)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{cfg} inflight={m} ms_per_block={dt / n * 1e3:.4f} blocks_per_s={n / dt:.1f}", flush=True)
        del exprs, opss, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
