"""The HIP path against the committed golden fixtures (tests/golden/*.npz; oracle-generated,
parity with the reference itself unpinned)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, f"{name}.npz"), allow_pickle=False)


def test_golden_sandwich_hip(dev):
    import torch
    from tneq_qc_amd.backends import BackendFactory
    from tneq_qc_amd.contractor import StrategyCompiler
    from tneq_qc_amd.core import QCTN
    d = _load("sandwich")
    q = QCTN(str(d["graph"]))
    be = BackendFactory.create_backend("hip", device="cuda:0", dtype="complex128")
    states = [np.array([1.0, 0.0], complex)] * 3
    mx = list(d["mx"])
    fn, name, _ = StrategyCompiler("balanced").compile(
        q, {"circuit_states_shapes": tuple(s.shape for s in states),
            "measure_shapes": tuple(m.shape for m in mx), "measure_is_matrix": True}, be)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    cores = {c: T(d[f"core_{i}"]) for i, c in enumerate(q.cores)}
    got = fn(cores, [T(s) for s in states], [T(m) for m in mx]).cpu().numpy()
    ref = d["expected"]
    assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max()


@pytest.mark.parametrize("dtype,tol", [("complex128", 1e-12), ("complex64", 1e-5)])
def test_golden_amplitude_hip(dev, dtype, tol):
    import torch
    from tneq_qc_amd.expression import HipContractExpression
    d = _load("amplitude")
    n = int(d["n_cores"])
    eq = str(d["equation"])
    ops = [torch.from_numpy(d[f"core_{i}"]).to(dev, getattr(torch, dtype)) for i in range(n)]
    expr = HipContractExpression(eq, *[tuple(o.shape) for o in ops], optimize="greedy")
    got = expr(*ops).cpu().numpy()
    ref = d["expected"]
    assert np.abs(got - ref).max() <= tol * np.abs(ref).max()


def test_golden_hermite_and_icdf_hip(dev):
    import torch
    from tneq_qc_amd import ops
    from oracle.data_ref import mx_weights
    d = _load("hermite")
    K = int(d["K"])
    x = torch.from_numpy(d["x"]).to(dev)
    phi, mx = ops.hermite_features(x, K, mx_weights(K), torch.complex128)
    assert np.abs(phi.cpu().numpy() - d["phi_c"]).max() <= 1e-13 * np.abs(d["phi_c"]).max()
    assert np.abs(mx.cpu().numpy() - d["mx_c"]).max() <= 1e-13 * np.abs(d["mx_c"]).max()
    phi, mx = ops.hermite_features(x.float(), K, mx_weights(K), torch.float32)
    assert np.abs(phi.cpu().numpy() - d["phi_f32"]).max() <= 2e-6 * np.abs(d["phi_f32"]).max()
    assert np.abs(mx.cpu().numpy() - d["mx_f32"]).max() <= 2e-6 * np.abs(d["mx_f32"]).max()
    e = _load("icdf")
    T = lambda a: torch.from_numpy(a).to(dev)
    got = ops.inverse_cdf_sample(T(e["density"]), T(e["grid"]), T(e["u"])).cpu().numpy()
    assert np.allclose(got, e["expected"], rtol=1e-9, atol=1e-9)
