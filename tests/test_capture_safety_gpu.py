"""Capture-safe teardown: the last reference to an expression -- its native
plans (arena, tables, hipGraphs) and its reverse-tree runtime (step plans + captured
CUDAGraphs) -- dropped INSIDE a caller's torch.cuda.graph capture.  HIP refuses
hipGraphExecDestroy / hipFree while a stream captures, so the releases are parked
(graphs.defer_release) and run at the next call outside the capture.  Checked: the capture
completes and replays the right values, the parked objects are released afterwards (nothing
left); tq_plan_destroy itself reports a refused HIP release instead of ignoring it and keeps
the plan for a retry (tq_plan.cpp plan_release)."""
import gc

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ops(torch, shapes, seed, req=False):
    rng = np.random.default_rng(seed)
    return [torch.tensor(rng.standard_normal(s) + 1j * rng.standard_normal(s), device="cuda",
                         requires_grad=req) for s in shapes]


def test_drop_expression_inside_user_capture(dev):
    import torch
    from tneq_qc_amd import graphs
    from tneq_qc_amd.expression import HipContractExpression
    eq, shapes = "ab,bc,cd->ad", [(8, 16), (16, 32), (32, 4)]
    # a forward-only expression whose plan has captured its own hipGraph (called twice), and a
    # differentiable one whose reverse-tree runtime has captured forward / backward graphs
    e_old = HipContractExpression(eq, *shapes)
    x_old = _ops(torch, shapes, 1)
    for _ in range(3):
        e_old(*x_old)
    e_grad = HipContractExpression(eq, *shapes)
    xg = _ops(torch, shapes, 2, req=True)
    for _ in range(3):
        out = e_grad(*xg)
        torch.autograd.grad(out.abs().sum(), xg)
    torch.cuda.synchronize()
    assert graphs.drain_deferred() == 0
    # the captured expression, warmed on the capture stream
    e_new = HipContractExpression(eq, *shapes)
    x_new = _ops(torch, shapes, 3)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            e_new(*x_new)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gc.collect()                     # no cyclic garbage of earlier tests left for the capture
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = e_new(*x_new)
        del e_old, e_grad          # last references: plans and runtime graphs die mid-capture,
        gc.collect()               # by refcount or (a cycle through the runtime) by a collection
        parked = graphs.deferred_count()
    assert parked >= 2, parked       # at least one plan handle and the runtime's graph dict
    torch.cuda.synchronize()
    x_new[0].mul_(2)                 # replay sees the new input values
    g.replay()
    torch.cuda.synchronize()
    ref = np.einsum(eq, *[t.cpu().numpy() for t in x_new])
    assert np.abs(out.cpu().numpy() - ref).max() <= 2e-5 * np.abs(ref).max()
    assert graphs.drain_deferred() == 0   # released now, outside the capture
    # the library is still healthy: a fresh expression after the drain
    e2 = HipContractExpression(eq, *shapes)
    ref2 = np.einsum(eq, *[t.cpu().numpy() for t in x_new])
    assert np.abs(e2(*x_new).cpu().numpy() - ref2).max() <= 2e-5 * np.abs(ref2).max()
    del g
