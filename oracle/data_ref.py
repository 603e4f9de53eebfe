"""ORACLE (test infrastructure only — never imported by the product path): numpy restatement of
EngineSiamese's measurement-data helpers.

  mx_weights(k_max)        engine_siamese.py:59-80    w_k = exp(-(log(2 pi)/2 + lgamma(k+1))/2)
  hermitenorm(n, x, dt)    engine_siamese.py:82-131   He_0 = 1, He_1 = x, He_i = x He_{i-1} - (i-1) He_{i-2}
  generate_data(x, K, ..)  engine_siamese.py:133-254  phi = (w * sqrt(exp(-x^2/2))) * He, Mx = conj(phi) (x) phi;
                           complex backend: float64 from the real part (:165-207);
                           real backend: the backend's precision (:212-254)
  inverse_cdf(d, grid, u)  engine_siamese.py:857-905  clamp >= 0, cumsum, / (total + 1e-10),
                           idx = min(#(cdf < u), G-2), linear interpolation on the grid
  sample(...)              engine_siamese.py:740-915  with a given sequence of uniform draws

Parity with the reference's own outputs is unpinned (importing the reference is denied,
SURVEY.md §8(c)); these restatements are pinned by known answers in tests/test_data_cpu.py
(closed-form He_k, orthonormality of phi_k, the inverse CDF of a uniform density).
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np


def mx_weights(k_max: int) -> np.ndarray:                                              # :59-80
    k = np.arange(k_max + 1, dtype=np.float64)
    log_factorial = np.array([math.lgamma(int(v) + 1) for v in k], dtype=np.float64)
    return np.exp(-0.5 * (0.5 * math.log(2 * math.pi) + log_factorial)).astype(np.float64)


def hermitenorm(n_max: int, x, dtype=np.float64) -> np.ndarray:                        # :82-131
    x = np.asarray(x, dtype=dtype)
    H = np.zeros((n_max + 1,) + x.shape, dtype=dtype)
    H[0] = 1.0
    if n_max >= 1:
        H[1] = x
        for i in range(2, n_max + 1):
            H[i] = x * H[i - 1] - (i - 1) * H[i - 2]
    return H


def generate_data(x, K: int, complex_backend: bool = True, real_dtype=np.float64):    # :133-254
    """(Mx_list, phi): Mx_list[i] is the (B, K, K) matrix batch of qubit i, phi is (B, D, K)."""
    x = np.asarray(x)
    if complex_backend:
        xr = np.asarray(np.real(x), dtype=np.float64)
        w = mx_weights(K - 1)[None, None, :K]
        H = hermitenorm(K - 1, xr)
        g = np.sqrt(np.exp(-np.square(xr) / 2.0))[..., None]
        phi = w * g * np.transpose(H, (1, 2, 0))
        Mx = np.einsum("bdk,bdl->bdkl", phi, phi)
    else:
        xr = np.asarray(np.real(x), dtype=real_dtype)
        w = mx_weights(K - 1)[:K].astype(real_dtype)[None, None, :]
        H = np.transpose(hermitenorm(K - 1, xr, real_dtype), (1, 2, 0))
        g = np.sqrt(np.exp(-np.square(xr) / 2))[..., None]
        phi = w * g * H
        Mx = np.einsum("bdk,bdl->bdkl", np.conj(phi), phi)
    return [Mx[:, i] for i in range(x.shape[1])], phi


def inverse_cdf(density, grid, u) -> np.ndarray:                                        # :857-905
    d = np.asarray(density)
    d = np.where(d < 0, np.zeros_like(d), d)
    cdf = np.cumsum(d, axis=1)
    cdf = cdf / (cdf[:, -1:] + 1e-10)
    uu = np.asarray(u, dtype=np.float32).reshape(-1).astype(cdf.dtype)
    G = cdf.shape[1]
    idx = np.minimum((cdf < uu[:, None]).sum(axis=1), G - 2)
    r = np.arange(cdf.shape[0])
    cl, cr = cdf[r, idx], cdf[r, idx + 1]
    g = np.asarray(grid, dtype=cdf.dtype)
    xl, xr = g[idx], g[idx + 1]
    frac = (uu - cl) / (cr - cl + 1e-10)
    return xl + frac * (xr - xl)


def sample(qctn, cores, states, num_samples: int, K: int, bounds, grid_size: int,
           uniforms: Sequence[np.ndarray]) -> np.ndarray:                               # :740-915
    """Sequential inverse-CDF sampling with the given per-qubit uniforms (complex backend).
    Measurements: the grid Mx on the current qubit, the sampled Mx on earlier qubits, the
    identity on later ones, as (S*G, K, K) batches; density = the engine's Born rule |res|^2."""
    from .greedy_ref import greedy_contract
    S, G, n = num_samples, grid_size, qctn.nqubits
    grid = np.linspace(bounds[0], bounds[1], G)
    Mx_grid = generate_data(grid[:, None], K)[0][0]
    ident = np.eye(K)
    persistent = [None] * n
    out = np.zeros((S, n))
    for q in range(n):
        mx = []
        for i in range(n):
            if i == q:
                m = np.broadcast_to(Mx_grid[None], (S, G, K, K))
            elif i < q:
                m = np.broadcast_to(persistent[i][:, None], (S, G, K, K))
            else:
                m = np.broadcast_to(ident, (S, G, K, K))
            mx.append(np.ascontiguousarray(m).reshape(S * G, K, K).astype(np.complex128))
        res = greedy_contract(qctn, cores, states, mx)
        dens = (np.abs(res) ** 2 if np.iscomplexobj(res) else res).reshape(S, G)
        y = inverse_cdf(dens, grid, uniforms[q])
        out[:, q] = y
        persistent[q] = generate_data(y[:, None], K)[0][0]
    return out
