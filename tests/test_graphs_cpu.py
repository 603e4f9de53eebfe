"""graphs.gc_paused: Python's cyclic GC is off inside a torch graph capture (a collection there can
run a finalizer that destroys another CUDAGraph, which HIP refuses while a stream is capturing:
found r04 as an abort of the GPU suite under pytest's fd capture) and restored after."""
import gc

import pytest


def test_gc_paused_disables_and_restores():
    from tneq_qc_amd.graphs import gc_paused
    assert gc.isenabled()
    with gc_paused():
        assert not gc.isenabled()
    assert gc.isenabled()
    with pytest.raises(RuntimeError):
        with gc_paused():
            raise RuntimeError("capture failed")
    assert gc.isenabled()          # restored on the error path too
    gc.disable()
    try:
        with gc_paused():
            assert not gc.isenabled()
        assert not gc.isenabled()  # a caller's disabled GC stays disabled
    finally:
        gc.enable()
