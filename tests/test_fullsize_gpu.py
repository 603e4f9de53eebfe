"""Full-size parity on the GPU through size-independent properties (BASELINE.json configs).

* C2 (30q depth-14, one amplitude): small enough for the oracle -> direct comparison.
* C3 / C4 (sliced, 2^16 / 2^20 amplitudes): the sliced + hoisted execution equals the unsliced
  contraction of the same network, every rank-shard of the slices sums to the full result, and
  the amplitudes of a unitary circuit satisfy sum |amp|^2 <= 1 (they are a sub-block of |psi>).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _expr_and_ops(task, dev, dtype, sliced=True):
    import torch
    from tneq_qc_amd.expression import HipContractExpression
    e = HipContractExpression(task.eq, *task.shapes, optimize=task.path,
                              slices=task.sliced if sliced else ())
    ops = [torch.from_numpy(o).to(dev, dtype) for o in task.operands]
    return e, ops


def test_c2_single_amplitude_vs_oracle(dev):
    import torch
    from oracle.contract_ref import contract as ref_contract
    from tneq_qc_amd.circuits import config_task
    t = config_task("C2")
    ref = ref_contract(t.eq, *t.operands, path=t.path)
    for dt, tol in ((torch.complex128, 1e-12), (torch.complex64, 2e-5)):
        e, ops = _expr_and_ops(t, dev, dt)
        got = e(*ops).cpu().numpy()
        assert abs(got - ref) / abs(ref) < tol


@pytest.mark.parametrize("cfg", ["C3", "C4"])
def test_sliced_equals_unsliced(dev, cfg):
    import torch
    from tneq_qc_amd.circuits import config_task
    t = config_task(cfg)
    e, ops = _expr_and_ops(t, dev, torch.complex64)
    sliced = e(*ops)
    e0, _ = _expr_and_ops(t, dev, torch.complex64, sliced=False)
    full = e0(*ops)
    err = (sliced - full).abs().max().item() / full.abs().max().item()
    assert err < 1e-4, err
    # 4-way shard of the slices accumulated == full sum
    acc = torch.zeros_like(full)
    for r in range(4):
        e(*ops, out=acc, slice_range=(r, e.n_slices, 4), accumulate=True)
    err2 = (acc - full).abs().max().item() / full.abs().max().item()
    assert err2 < 1e-4, err2
    p = (full.abs() ** 2).sum().item()
    assert 0.0 < p <= 1.0 + 1e-4
