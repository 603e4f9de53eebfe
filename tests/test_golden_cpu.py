"""The oracle reproduces the committed golden fixtures (tests/golden/*.npz, written by
tests/golden/make_golden.py): any drift of the CPU restatement shows here.  Parity with the
reference itself is unpinned; these fixtures pin the oracle in time."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, f"{name}.npz"), allow_pickle=False)


def _cores(d, q):
    return {c: d[f"core_{i}"] for i, c in enumerate(q.cores)}


def test_golden_sandwich_oracle():
    from oracle.greedy_ref import greedy_contract
    from oracle.qctn_ref import QCTNRef
    d = _load("sandwich")
    q = QCTNRef(str(d["graph"]))
    assert len(q.cores) == int(d["n_cores"])
    out = greedy_contract(q, _cores(d, q), [np.array([1.0, 0.0], complex)] * 3, list(d["mx"]))
    assert np.allclose(out, d["expected"], rtol=1e-13, atol=1e-15)


def test_golden_amplitude_oracle():
    from oracle.contract_ref import contract
    from oracle.qctn_ref import QCTNRef, build_core_only_expression
    d = _load("amplitude")
    q = QCTNRef(str(d["graph"]))
    eq, _ = build_core_only_expression(q)
    assert eq == str(d["equation"])
    out = contract(eq, *[_cores(d, q)[c] for c in q.cores])
    assert np.allclose(out, d["expected"], rtol=1e-13, atol=1e-15)
    assert abs(np.vdot(out, out).real - 2 ** 6) < 1e-9   # unitary cores: ||U||_F^2 = 2^n


def test_golden_hermite_and_icdf_oracle():
    from oracle.data_ref import generate_data, inverse_cdf
    d = _load("hermite")
    K = int(d["K"])
    mc, pc = generate_data(d["x"], K)
    assert np.array_equal(pc, d["phi_c"]) and np.array_equal(np.stack(mc, 1), d["mx_c"])
    mr, pr = generate_data(d["x"], K, complex_backend=False, real_dtype=np.float32)
    assert np.array_equal(pr, d["phi_f32"]) and np.array_equal(np.stack(mr, 1), d["mx_f32"])
    e = _load("icdf")
    assert np.array_equal(inverse_cdf(e["density"], e["grid"], e["u"]), e["expected"])
