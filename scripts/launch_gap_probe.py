#!/usr/bin/env python3
"""Probe: the cost per dependent kernel launch on this box — 200 tiny dependent kernels (an
in-place add on 64 KiB) issued eagerly on one stream and replayed from a captured hipGraph;
time per kernel = the launch gap + a ~2 us kernel.
    python scripts/launch_gap_probe.py"""
import json

import torch

dev = torch.device("cuda:0")
x = torch.zeros(16384, device=dev)
N = 200


def chain():
    for _ in range(N):
        x.add_(1.0)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3 / N   # us per kernel


eager = timed(chain)
s = torch.cuda.Stream(dev)
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    chain()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    chain()
graph = timed(g.replay)
print(json.dumps({"us_per_kernel_eager": eager, "us_per_kernel_graph": graph, "kernels": N}), flush=True)
