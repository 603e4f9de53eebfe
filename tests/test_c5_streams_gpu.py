"""C5 training candidates on separate HIP streams (scripts/c5_bench.py gpu_step(streams=...)):
the candidates are independent fits, so running each on its own stream must give exactly the
results of running them one after another -- same losses, same parameters after the SGDG steps
(complex128, <= 1e-12 relative)."""
import importlib.util
import os
import random

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c5():
    spec = importlib.util.spec_from_file_location("c5_bench", os.path.join(ROOT, "scripts", "c5_bench.py"))
    cb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cb)
    return cb


def test_candidates_on_streams_equal_sequential(dev):
    import torch
    cb = _c5()
    runs = []
    for use_streams in (False, True):
        random.seed(0)   # the SGDG retraction draw
        target, cands = cb.setup(dev)
        streams = [torch.cuda.Stream(dev) for _ in cands] if use_streams else None
        losses = []
        for _ in range(3):
            losses.append([float(l.detach()) for l in cb.gpu_step(target, cands, streams)])
        torch.cuda.synchronize()
        runs.append((losses, [[p.detach().clone() for p in c[1]] for c in cands]))
    (l0, p0), (l1, p1) = runs
    for a, b in zip(l0, l1):
        for x, y in zip(a, b):
            assert abs(x - y) <= 1e-12 * max(1.0, abs(x))
    for ca, cb_ in zip(p0, p1):
        for a, b in zip(ca, cb_):
            assert (a - b).abs().max().item() <= 1e-12 * max(1.0, a.abs().max().item())


def test_graphed_steps_equal_eager(dev):
    """Forward + loss + backward of every candidate captured once as a hipGraph
    (tneq_qc_amd.graphs.capture_step) and replayed per step, SGDG eager: the same losses and
    parameters as the eager steps (complex128, <= 1e-12 relative), candidates on streams."""
    import torch
    cb = _c5()
    runs = []
    for graphed in (False, True):
        random.seed(0)
        target, cands = cb.setup(dev)
        streams = [torch.cuda.Stream(dev) for _ in cands]
        graphs = cb.capture(target, cands, dev) if graphed else None
        losses = []
        for _ in range(3):
            losses.append([float(l.detach()) for l in cb.gpu_step(target, cands, streams, graphs)])
        torch.cuda.synchronize()
        runs.append((losses, [[p.detach().clone() for p in c[1]] for c in cands]))
    (l0, p0), (l1, p1) = runs
    for a, b in zip(l0, l1):
        for x, y in zip(a, b):
            assert abs(x - y) <= 1e-12 * max(1.0, abs(x))
    for ca, cb_ in zip(p0, p1):
        for a, b in zip(ca, cb_):
            assert (a - b).abs().max().item() <= 1e-12 * max(1.0, a.abs().max().item())
