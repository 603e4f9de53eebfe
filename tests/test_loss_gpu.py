"""The fused fidelity loss (ops.fidelity_loss: tq_fidelity_forward / tq_fidelity_backward) against
the reference's torch expression (symmetry_breaking_quantum.py:224-228: vdot, abs()**2,
clamp_min(1e-12), 1 - num/den) with torch autograd, on the same device.  Tolerances: complex128
1e-12, complex64 2e-5 (float64 accumulation vs torch's float32 dots), relative."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ref(out, tgt):
    import torch
    o, t = out.reshape(-1), tgt.reshape(-1)
    num = torch.vdot(t, o).abs() ** 2
    den = (torch.vdot(t, t).real * torch.vdot(o, o).real).clamp_min(1e-12)
    return 1.0 - num / den


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
@pytest.mark.parametrize("n", [1, 7, 4096, 65536, 300001])
def test_fidelity_loss_and_gradient_match_torch(dev, dtype, n):
    import torch
    from tneq_qc_amd.ops import fidelity_loss
    dt = getattr(torch, dtype)
    rng = np.random.default_rng(n)
    tol = 1e-12 if dtype == "complex128" else 2e-5
    t = torch.tensor(rng.standard_normal(n) + 1j * rng.standard_normal(n), dtype=dt, device=dev)
    # an output correlated with the target (fidelity well inside (0, 1))
    o0 = 0.7 * t + 0.3 * torch.tensor(rng.standard_normal(n) + 1j * rng.standard_normal(n), dtype=dt, device=dev)
    a = o0.clone().requires_grad_(True)
    b = o0.clone().requires_grad_(True)
    la = fidelity_loss(a, t)
    lb = _ref(b, t)
    assert la.dtype == lb.dtype and la.shape == lb.shape
    assert abs(la.item() - lb.item()) <= tol * max(1.0, abs(lb.item()))
    (3.0 * la).backward()     # an upstream gradient other than 1
    (3.0 * lb).backward()
    # the gradient's two terms are each ~ 2 |<t,o>| max|t| / (<t,t> <o,o>) (they cancel at n = 1,
    # where the fidelity is identically 1): errors are measured against that magnitude
    with torch.no_grad():
        ov = torch.vdot(t, o0).abs().item()
        term = 3.0 * 2.0 * ov * t.abs().max().item() / (torch.vdot(t, t).real.item() * torch.vdot(o0, o0).real.item())
    assert (a.grad - b.grad).abs().max().item() <= tol * 10 * term


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_fidelity_loss_clamped_denominator(dev, dtype):
    """<t,t> <o,o> below 1e-12: den is the constant 1e-12 and <o,o> gets no gradient (the
    clamp's), as in torch."""
    import torch
    from tneq_qc_amd.ops import fidelity_loss
    dt = getattr(torch, dtype)
    rng = np.random.default_rng(1)
    t = torch.tensor(rng.standard_normal(64) + 1j * rng.standard_normal(64), dtype=dt, device=dev)
    o0 = 1e-9 * torch.tensor(rng.standard_normal(64) + 1j * rng.standard_normal(64), dtype=dt, device=dev)
    assert (torch.vdot(t, t).real * torch.vdot(o0, o0).real).item() < 1e-12   # the clamp is active
    a = o0.clone().requires_grad_(True)
    b = o0.clone().requires_grad_(True)
    la, lb = fidelity_loss(a, t), _ref(b, t)
    assert abs(la.item() - lb.item()) <= 1e-6 * max(1.0, abs(lb.item()))
    la.backward()
    lb.backward()
    scale = b.grad.abs().max().item()
    assert (a.grad - b.grad).abs().max().item() <= 1e-6 * scale


def test_fidelity_loss_rejects_bad_operands(dev):
    import torch
    from tneq_qc_amd.ops import fidelity_loss
    t = torch.zeros(8, dtype=torch.complex128, device=dev)
    with pytest.raises(ValueError):
        fidelity_loss(torch.zeros(8, dtype=torch.float64, device=dev), t)
    with pytest.raises(ValueError):
        fidelity_loss(torch.zeros(9, dtype=torch.complex128, device=dev), t)
