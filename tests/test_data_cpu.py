"""The measurement-data oracle (oracle/data_ref.py) pinned by known answers, the C-ABI argument
checks of the data kernels (no compute), and the engine's host-side pieces (CPU only)."""
import math

import numpy as np
import pytest

from oracle.data_ref import generate_data, hermitenorm, inverse_cdf, mx_weights


def test_hermite_closed_forms():
    x = np.linspace(-3, 3, 13)
    H = hermitenorm(4, x)
    assert np.allclose(H[0], 1) and np.allclose(H[1], x)
    assert np.allclose(H[2], x ** 2 - 1)
    assert np.allclose(H[3], x ** 3 - 3 * x)
    assert np.allclose(H[4], x ** 4 - 6 * x ** 2 + 3)
    assert hermitenorm(0, x).shape == (1, 13)


def test_weights_and_orthonormality():
    """phi_k(x) = w_k e^{-x^2/4} He_k(x) is orthonormal on R, since
    int He_k He_l e^{-x^2/2} dx = sqrt(2 pi) k! delta_kl (engine_siamese.py:59-80 weights)."""
    w = mx_weights(6)
    assert np.isclose(w[0], (2 * math.pi) ** -0.25)
    assert np.allclose(w[1:] / w[:-1], 1 / np.sqrt(np.arange(1, 7)))
    x = np.linspace(-12, 12, 20001)
    Mx, phi = generate_data(x[:, None], 6)
    gram = (phi[:, 0, :, None] * phi[:, 0, None, :]).sum(0) * (x[1] - x[0])
    assert np.abs(gram - np.eye(6)).max() < 1e-9
    assert len(Mx) == 1 and Mx[0].shape == (20001, 6, 6)
    assert np.allclose(Mx[0][:, 2, 3], phi[:, 0, 2] * phi[:, 0, 3])


def test_real_path_keeps_backend_precision():
    x = np.array([[0.5, -1.25], [2.0, 3.5]], np.float32)
    Mx, phi = generate_data(x, 5, complex_backend=False, real_dtype=np.float32)
    assert phi.dtype == np.float32 and Mx[0].dtype == np.float32
    M64, p64 = generate_data(x.astype(np.float64), 5)
    assert np.allclose(phi, p64, rtol=1e-5, atol=1e-7)


def test_inverse_cdf_known_answers():
    G = 101
    grid = np.linspace(0.0, 1.0, G)
    u = np.array([0.05, 0.25, 0.5, 0.75, 0.95], np.float32)
    y = inverse_cdf(np.ones((5, G)), grid, u)
    # cdf_i = (i+1)/G, and the reference interpolates on the cell [idx, idx+1] with
    # idx = #(cdf < u): the linear inverse maps u to grid position (u G - 1) / (G - 1)
    assert np.allclose(y, (u.astype(np.float64) * G - 1) / (G - 1), atol=1e-9)
    # negatives are clamped to 0; an all-zero row extrapolates from the last cell (quirk kept)
    d = np.ones((2, G))
    d[1, ::2] = -1.0
    d0 = d.copy()
    d0[1, ::2] = 0.0
    assert np.array_equal(inverse_cdf(d, grid, u[:2]), inverse_cdf(d0, grid, u[:2]))
    z = inverse_cdf(np.zeros((1, G)), grid, np.array([0.5], np.float32))
    assert np.isclose(z[0], grid[G - 2] + 0.5 / 1e-10 * (grid[G - 1] - grid[G - 2]))


def test_data_abi_rejects_bad_arguments():
    """Argument checks of tq_hermite_features / tq_inverse_cdf_sample run before any launch."""
    import ctypes
    from tneq_qc_amd import _lib
    L = _lib.lib()
    w = (ctypes.c_double * 4)(1, 1, 1, 1)
    assert L.tq_hermite_features(_lib.TQ_C64, 4, 0, None, w, None, None, None) == _lib.TQ_ERR_INVALID
    assert L.tq_hermite_features(_lib.TQ_C64, 4, 129, None, w, None, None, None) == _lib.TQ_ERR_INVALID
    assert L.tq_hermite_features(9, 4, 2, None, w, None, None, None) == _lib.TQ_ERR_INVALID
    assert L.tq_hermite_features(_lib.TQ_C64, 0, 2, None, w, None, ctypes.c_void_p(1), None) == _lib.TQ_OK
    assert L.tq_inverse_cdf_sample(_lib.TQ_C64, 1, 10, None, 10, None, None, None, 1, None) == _lib.TQ_ERR_INVALID
    assert L.tq_inverse_cdf_sample(_lib.TQ_F64, 1, 1, None, 1, None, None, None, 1, None) == _lib.TQ_ERR_INVALID
    assert L.tq_inverse_cdf_sample(_lib.TQ_F64, 1, 8193, None, 8193, None, None, None, 1, None) == _lib.TQ_ERR_INVALID
    assert L.tq_inverse_cdf_sample(_lib.TQ_F64, 0, 10, None, 10, None, None, None, 1, None) == _lib.TQ_OK


def test_ops_wrappers_require_device_tensors():
    import torch
    from tneq_qc_amd import ops
    with pytest.raises(ValueError):
        ops.hermite_features(torch.zeros(3, 2), 4, mx_weights(4), torch.complex128)
    with pytest.raises(ValueError):
        ops.inverse_cdf_sample(torch.zeros(3, 5), torch.zeros(5), torch.zeros(3))
