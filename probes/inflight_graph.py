"""Two blocks in flight, launched as ONE captured graph per pair of blocks (both plans' executes on
two forked streams inside a torch CUDA graph capture; the plans enqueue into the capture) against
the bench's form (each plan's own graph on its own stream, one launch per block).

    python probes/inflight_graph.py [C4] [n]
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
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    dev = torch.device("cuda:0")
    base = config_task(cfg)
    slots = []
    for i in range(2):
        t = with_batch(base, i)
        e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
        ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in t.operands]
        slots.append((e, ops, torch.empty(e.out_shape, dtype=torch.complex64, device=dev), torch.cuda.Stream(dev)))
    # the bench's form
    def step(k):
        e, ops, out, s = slots[k % 2]
        with torch.cuda.stream(s):
            e(*ops, out=out)
    for k in range(10):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(n):
        step(k)
    torch.cuda.synchronize()
    a = (time.perf_counter() - t0) / n * 1e3
    ref = [s[2].clone() for s in slots]
    # one graph per pair
    main_s = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=main_s):
        cur = torch.cuda.current_stream()
        for e, ops, out, s in slots:
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                e(*ops, out=out)
        for e, ops, out, s in slots:
            cur.wait_stream(s)
    torch.cuda.synchronize()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    ok = all(torch.allclose(s[2], r, rtol=0, atol=0) or torch.equal(s[2], r) for s, r in zip(slots, ref))
    t0 = time.perf_counter()
    for _ in range(n // 2):
        g.replay()
    torch.cuda.synchronize()
    b = (time.perf_counter() - t0) / (2 * (n // 2)) * 1e3
    print(f"{cfg} per block: streams {a:.4f} ms, pair graph {b:.4f} ms, same result {ok}", flush=True)


if __name__ == "__main__":
    main()
