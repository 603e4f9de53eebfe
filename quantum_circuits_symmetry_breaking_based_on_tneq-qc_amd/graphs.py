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


# Releases deferred while a stream capture is in progress: HIP refuses hipGraphExecDestroy /
# hipFree / hipStreamDestroy during a (global-mode) capture, so an object whose last reference
# drops inside a caller's `torch.cuda.graph` capture -- a plan, a reverse-tree runtime with its
# CUDAGraphs -- parks its resources here; they are released at the next call that runs outside a
# capture (drain_deferred: plan creation / execution, the end of our own capture sites, exit).
_DEFERRED: list = []


def capturing() -> bool:
    """True while the current stream captures (a caller's torch.cuda.graph block)."""
    try:
        return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
    except Exception:   # interpreter shutdown
        return False


def defer_release(obj) -> None:
    """Keep `obj` (a plan handle wrapper or any object holding HIP resources) alive until the
    next drain outside a capture."""
    _DEFERRED.append(obj)


def drain_deferred() -> int:
    """Release what was parked during captures (outside a capture only); returns how many
    objects are still parked."""
    if not _DEFERRED or capturing():
        return len(_DEFERRED)
    items = _DEFERRED[:]
    del _DEFERRED[:]
    for it in items:
        rel = getattr(it, "release_now", None)
        if rel is not None:
            rel()                  # may park itself again if HIP still refuses
    del items                      # the rest (e.g. CUDAGraphs) die here
    return len(_DEFERRED)


def deferred_count() -> int:
    return len(_DEFERRED)


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
    drain_deferred()
    return g, loss
