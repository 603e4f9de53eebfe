"""Pre-split boundary-GEMM operands on the GPU (opt-in path) (tq_gemm.hip SplitPre, tq_sweep2.hip f16_terms,
tq_plan.cpp Op::ps_cand): the per-slice sweep ops that store the two operands of the C3 / C4g
boundary GEMM write them as the f16 terms (h, l) of their values scaled by 2^sc, sc predicted
from the previous slice's operand max; the GEMM checks the true max against the window
(max * 2^sc in [2^0, 2^15)) and a slice outside it is re-run on the split path.

* the pre-split path is the one that runs (plan query n_presplit, no fallbacks once the
  prediction is warm) and equals the split path (2e-5 of max|amp|; both are within 2e-5 of the
  exact contraction) and the oracle on a benchmarked slice;
* a scale pushed 30 binades either way (library knob presplit_bias) puts every slice outside
  the window: every slice is re-run and the result is unchanged.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 2e-5


def _lib():
    from tneq_qc_amd import _lib as lib
    return lib.lib()


@pytest.fixture(autouse=True)
def presplit_on():
    """The pre-split path is opt-in (tq_library_set("gemm_presplit", 1) / TQ_GEMM_PRESPLIT=1) and
    runs on the 4-multiplication f16 tile (gemm_f16_var 0; the default is the Gauss tile)."""
    L = _lib()
    prev = L.tq_library_query(b"gemm_presplit")
    prev_var = L.tq_library_query(b"gemm_f16_var")
    assert L.tq_library_set(b"gemm_presplit", 1) == 0
    assert L.tq_library_set(b"gemm_f16_var", 0) == 0
    yield
    L.tq_library_set(b"gemm_presplit", prev)
    L.tq_library_set(b"gemm_f16_var", prev_var)


def _expr(cfg, dev):
    import torch
    from tneq_qc_amd.circuits import config_task
    from tneq_qc_amd.expression import HipContractExpression
    t = config_task(cfg)
    e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
    ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in t.operands]
    return t, e, ops


def _split_path(cfg, dev, slice_range=None):
    L = _lib()
    assert L.tq_library_set(b"gemm_presplit", 0) == 0
    try:
        _, e, ops = _expr(cfg, dev)
        out = e(*ops, slice_range=slice_range) if slice_range else e(*ops)
        assert e.plan(out.dtype).query("presplit_fallbacks") == 0
        return out
    finally:
        L.tq_library_set(b"gemm_presplit", 1)


# C4g's boundary GEMM takes producer-written planes instead (tq_gemmp.hip; test_fullsize_gpu
# test_planes_gemm_equals_split_kernel): its plan has no pre-split candidate
@pytest.mark.parametrize("cfg,rng", [("C3", None), ("C3", (0, 3, 1))])
def test_presplit_runs_and_matches_split_path(dev, cfg, rng):
    import torch
    assert _lib().tq_library_query(b"gemm_presplit") == 1
    _, e, ops = _expr(cfg, dev)
    run = (lambda: e(*ops, slice_range=rng)) if rng else (lambda: e(*ops))
    first = run()
    p = e.plan(torch.complex64)
    assert p.query("n_presplit") == 1
    f0 = p.query("presplit_fallbacks")
    got = run()   # warm prediction: no slice leaves its window
    assert p.query("presplit_fallbacks") == f0
    ref = _split_path(cfg, dev, rng)
    amax = ref.abs().max().item()
    for out in (first, got):
        err = (out - ref).abs().max().item() / amax
        assert err < TOL, (cfg, err)


def test_presplit_slice_vs_oracle(dev):
    """C3 slice 37 on the pre-split path against the oracle's exact contraction of it."""
    from oracle.contract_ref import contract as ref_contract, sliced_operands
    t, e, ops = _expr("C3", dev)
    e(*ops, slice_range=(36, 37, 1))        # the prediction for slice 37 comes from slice 36
    got = e(*ops, slice_range=(37, 38, 1)).cpu().numpy()
    eq, sops = sliced_operands(t.eq, t.operands, t.sliced, 37)
    ref = ref_contract(eq, *sops, path=t.path)
    amax = np.abs(ref).max()
    assert np.abs(got - ref).max() / amax < TOL


@pytest.mark.parametrize("bias", [30, -30])
def test_presplit_window_fallback(dev, bias):
    import torch
    L = _lib()
    ref = _split_path("C3", dev)
    assert L.tq_library_set(b"presplit_bias", bias) == 0
    try:
        _, e, ops = _expr("C3", dev)
        got = e(*ops)
        p = e.plan(torch.complex64)
        assert p.query("presplit_fallbacks") == e.n_slices
        acc = torch.zeros_like(got)
        for r in range(2):   # shards accumulated into one buffer: re-run slices accumulate too
            e(*ops, out=acc, slice_range=(r, e.n_slices, 2), accumulate=True)
        assert p.query("presplit_fallbacks") == 2 * e.n_slices
    finally:
        L.tq_library_set(b"presplit_bias", 0)
    amax = ref.abs().max().item()
    assert (got - ref).abs().max().item() / amax < TOL
    assert (acc - ref).abs().max().item() / amax < TOL
