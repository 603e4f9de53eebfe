"""Whole training steps as hipGraphs.

The reference's training loop (symmetry_breaking_quantum.py:196-238, engine_siamese.py:351-554)
runs forward, loss and backward eagerly every step: on the HIP engine that is ~100 dependent
small launches per candidate-step, each issued from Python (the C5 line is host-issue bound).
`capture_step` records forward + loss + backward once into a torch.cuda.CUDAGraph (a hipGraph on
ROCm) on a stream of its own; every replay re-executes all of it on the current parameter values
(they are updated in place by the optimizer) and leaves the gradients in the parameters' .grad
tensors (static graph memory).  The optimizer step stays eager: SGDG's host-side random draw
(stiefel_optimizer_complex.py:111-113) decides per step and per parameter whether the
retraction runs, exactly as in the reference.
"""
from __future__ import annotations

import contextlib
import gc
from typing import Callable, Sequence, Tuple

import torch


@contextlib.contextmanager
def gc_paused():
    """Python's cyclic GC off for the duration (wrap a whole ``torch.cuda.graph`` capture in it).
    A collection triggered by an allocation inside a capture can run a finalizer that destroys
    another CUDAGraph (hipGraphExecDestroy), which HIP refuses while a stream is capturing: the
    refusal is raised inside ~CUDAGraph and terminates the process.  torch's capture context
    still runs its explicit gc.collect() before the capture begins."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def capture_step(step_fn: Callable[[], torch.Tensor], params: Sequence[torch.Tensor],
                 device: torch.device, warmup: int = 2) -> Tuple["torch.cuda.CUDAGraph", torch.Tensor]:
    """`step_fn()` runs forward + loss + ``loss.backward()`` and returns the loss.  Returns the
    captured graph and its (static) loss tensor.  Warmup runs on the capture stream first, so
    every plan, runtime buffer and workspace the step uses exists before capture; the parameters
    are not modified (no optimizer step inside).  After capture the parameters' ``.grad`` are the
    graph's gradient outputs: do not reset them (``zero_grad``) between replays."""
    s = torch.cuda.Stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        for _ in range(warmup):
            for p in params:
                p.grad = None
            step_fn()
    torch.cuda.current_stream(device).wait_stream(s)
    torch.cuda.synchronize(device)
    for p in params:
        p.grad = None
    g = torch.cuda.CUDAGraph()
    with gc_paused(), torch.cuda.graph(g, stream=s):
        loss = step_fn()
    torch.cuda.synchronize(device)
    return g, loss
