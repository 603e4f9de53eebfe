#!/usr/bin/env python3
"""Writes the golden fixtures of tests/golden/ from the CPU oracle (oracle/), with fixed seeds.

The fixtures are data (inputs + expected outputs), not reference code.  Importing or running the
reference (tneq_qc) is denied here, so the expected outputs come from the
oracle's restatement and parity with the reference itself stays unpinned; the fixtures freeze
the oracle's answers, so the CPU suite notices any drift of the restatement
(tests/test_golden_cpu.py) and the GPU suite compares the HIP path with fixed numbers
(tests/test_golden_gpu.py).

  sandwich.npz   3-qubit brick wall (2 cells), Haar cores (seed 7), |0> states, random complex
                 3-D Mx (B = 4): GreedyStrategy's raw result (oracle/greedy_ref.py)
  amplitude.npz  6-qubit, 3-cell brick wall, core-only tensor (2^12 entries) (oracle/contract_ref.py)
  hermite.npz    x (9, 3), K = 6: phi and Mx of the complex (float64) and float32 branches
                 (oracle/data_ref.py)
  icdf.npz       density (8, 64) with an empty row and negative entries, grid, u -> draws
                 (oracle/data_ref.py)

Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle.contract_ref import contract  # noqa: E402
from oracle.data_ref import generate_data, inverse_cdf  # noqa: E402
from oracle.greedy_ref import greedy_contract  # noqa: E402
from oracle.qctn_ref import (QCTNRef, build_brick_wall_IM, build_core_only_expression,  # noqa: E402
                             incidence_to_graph, random_cores)


def _cores_arrays(q, cores):
    return {f"core_{i}": cores[c] for i, c in enumerate(q.cores)}


def sandwich():
    g = incidence_to_graph(build_brick_wall_IM(3, 2))
    q = QCTNRef(g)
    cores = random_cores(q, 7)
    rng = np.random.default_rng(8)
    states = [np.array([1.0, 0.0], complex) for _ in range(3)]
    mx = [rng.standard_normal((4, 2, 2)) + 1j * rng.standard_normal((4, 2, 2)) for _ in range(3)]
    out = greedy_contract(q, cores, states, mx)
    return dict(graph=np.array(g), n_cores=np.array(len(q.cores)), mx=np.stack(mx),
                expected=np.asarray(out), **_cores_arrays(q, cores))


def amplitude():
    g = incidence_to_graph(build_brick_wall_IM(6, 3))
    q = QCTNRef(g)
    cores = random_cores(q, 9)
    eq, _ = build_core_only_expression(q)
    out = contract(eq, *[cores[c] for c in q.cores])
    return dict(graph=np.array(g), n_cores=np.array(len(q.cores)), equation=np.array(eq),
                expected=out, **_cores_arrays(q, cores))


def hermite():
    rng = np.random.default_rng(12)
    x = (rng.standard_normal((9, 3)) * 1.7).astype(np.float32).astype(np.float64)
    mc, pc = generate_data(x, 6, complex_backend=True)
    mr, pr = generate_data(x, 6, complex_backend=False, real_dtype=np.float32)
    return dict(x=x, K=np.array(6), phi_c=pc, mx_c=np.stack(mc, 1), phi_f32=pr, mx_f32=np.stack(mr, 1))


def icdf():
    rng = np.random.default_rng(13)
    d = rng.random((8, 64)) ** 3
    d[2] = 0.0
    d[5, ::4] = -0.5
    grid = np.linspace(-4.0, 4.0, 64)
    u = rng.random(8).astype(np.float32)
    return dict(density=d, grid=grid, u=u, expected=inverse_cdf(d, grid, u))


MAKERS = {"sandwich": sandwich, "amplitude": amplitude, "hermite": hermite, "icdf": icdf}


if __name__ == "__main__":
    for name, fn in MAKERS.items():
        path = os.path.join(HERE, f"{name}.npz")
        np.savez(path, **fn())
        print(path, os.path.getsize(path), "bytes")
