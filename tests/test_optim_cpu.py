"""The SGDG oracle (oracle/optim_ref.py, restating stiefel_optimizer_complex.py:77-176) on
known answers: zero gradient with zero momentum leaves the row-normalised parameter, the Cayley
step keeps a unitary core unitary, the 1-in-101 retraction draw follows Python's `random`, and
the SGD branch (rows > cols) applies weight decay / momentum / nesterov as torch.optim.SGD."""
import random

import numpy as np
import pytest


def _unitary(rng, n=4, dtype=np.complex128):
    q, r = np.linalg.qr(rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n)))
    return (q * (np.diag(r) / np.abs(np.diag(r)))[None, :]).astype(dtype)


def test_zero_gradient_is_a_fixed_point_of_the_normalised_parameter():
    from oracle.optim_ref import sgdg_step, unit
    rng = np.random.default_rng(0)
    p = (rng.standard_normal((2, 2, 2, 2)) + 1j * rng.standard_normal((2, 2, 2, 2))).astype(np.complex128)
    want = unit(p.reshape(4, 4))[0].reshape(p.shape)
    g = np.zeros_like(p)
    random.seed(3)
    sgdg_step([p], [g], {}, lr=0.1, momentum=0.9, stiefel=True)
    np.testing.assert_allclose(p, want, atol=1e-14)


@pytest.mark.parametrize("dtype,tol", [(np.complex128, 1e-12), (np.complex64, 2e-5)])
def test_cayley_step_keeps_unitary_cores_unitary(dtype, tol):
    from oracle.optim_ref import sgdg_step
    rng = np.random.default_rng(1)
    ps = [_unitary(rng, dtype=dtype).reshape(2, 2, 2, 2) for _ in range(3)]
    gs = [(rng.standard_normal((2, 2, 2, 2)) + 1j * rng.standard_normal((2, 2, 2, 2))).astype(dtype)
          for _ in range(3)]
    state = {}
    random.seed(11)
    for _ in range(3):
        sgdg_step(ps, [g.copy() for g in gs], state, lr=0.05, momentum=0.9, stiefel=True)
    for p in ps:
        u = p.reshape(4, 4)
        assert p.dtype == dtype
        np.testing.assert_allclose(u @ u.conj().T, np.eye(4), atol=tol)
    assert all(state[i]["momentum_buffer"].shape == (4, 4) for i in range(3))


def test_retraction_draw_follows_python_random():
    from oracle import optim_ref
    first = lambda s: (random.seed(s), random.randint(1, 101))[1]
    hit = next(s for s in range(10000) if first(s) == 1)
    miss = next(s for s in range(10000) if first(s) != 1)
    rng = np.random.default_rng(2)
    p = rng.standard_normal((2, 2, 2, 2)) + 1j * rng.standard_normal((2, 2, 2, 2))
    called = []
    orig = optim_ref.qr_retraction
    optim_ref.qr_retraction = lambda x: (called.append(1), orig(x))[1]
    try:
        for seed, want in ((hit, 1), (miss, 0)):
            called.clear()
            random.seed(seed)
            optim_ref.sgdg_step([p.copy()], [np.zeros_like(p)], {}, lr=0.1, stiefel=True)
            assert len(called) == want
    finally:
        optim_ref.qr_retraction = orig
    q = orig(p.reshape(4, 4))   # rows orthonormal
    np.testing.assert_allclose(q @ q.conj().T, np.eye(4), atol=1e-12)


def test_sgd_branch_matches_torch_sgd():
    import torch
    from oracle.optim_ref import sgdg_step
    rng = np.random.default_rng(3)
    p = rng.standard_normal((4, 2))          # rows 4 > cols 2 -> SGD branch even with stiefel=True
    gs = [rng.standard_normal((4, 2)) for _ in range(3)]
    tp = torch.tensor(p.copy(), requires_grad=True)
    opt = torch.optim.SGD([tp], lr=0.1, momentum=0.9, dampening=0.0, weight_decay=0.01, nesterov=True)
    state = {}
    for g in gs:
        sgdg_step([p], [g.copy()], state, lr=0.1, momentum=0.9, weight_decay=0.01, nesterov=True,
                  stiefel=True)
        tp.grad = torch.tensor(g.copy())
        opt.step()
    np.testing.assert_allclose(p, tp.detach().numpy(), atol=1e-14)
