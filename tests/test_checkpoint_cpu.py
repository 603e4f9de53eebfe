"""Host-side pieces of the plugin surface that need no GPU:

* the safetensors core format of QCTN.save_cores / load_cores / from_pretrained
  (tneq_qc/core/qctn.py:902-983): keys core_{name} for real cores, core_{name}_real/_imag for
  complex ones, value = tensor * scale for TNTensor cores, loaded cores become auto-scaled
  TNTensors (tn_tensor.py:67-85), strict / non-strict missing keys, metadata returned as the
  reference returns it;
* HipTreeStrategy.check_compatibility: general, as GreedyStrategy's (greedy_strategy.py:35-39).

The backend here is a minimal host stub (numpy arrays, the three ComputeBackend methods QCTN's
checkpoint code calls); the GPU suite repeats the round trip through BackendHIP.
"""
import numpy as np
import pytest


class _HostBackend:
    """torch CPU tensors (TNTensor's auto_scale uses tensor methods)."""

    def convert_to_tensor(self, a):
        import torch
        return torch.as_tensor(np.asarray(a))

    def tensor_to_numpy(self, t):
        import torch
        return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)

    def get_backend_name(self):
        return "host-stub"

    def init_random_core(self, shape):
        # QCTN(graph, backend) initialises cores at construction (qctn.py:724-760)
        import torch
        return torch.as_tensor(np.linalg.qr(np.random.default_rng(0).standard_normal(shape))[0])


def _qctn(n=3, cells=2):
    from tneq_qc_amd.circuits import build_brick_wall_IM, incidence_to_graph
    from tneq_qc_amd.core import QCTN
    g = incidence_to_graph(build_brick_wall_IM(n, cells))
    return g, QCTN(g, backend=_HostBackend())


def _cores(q, cplx, seed=0):
    rng = np.random.default_rng(seed)
    out = {}
    for c in q.cores:
        shp = q.core_shape(c)
        a = rng.standard_normal(shp)
        if cplx:
            a = a + 1j * rng.standard_normal(shp)
        out[c] = a
    return out


@pytest.mark.parametrize("cplx", [False, True])
def test_safetensors_keys_and_round_trip(tmp_path, cplx):
    from safetensors.numpy import load_file
    from tneq_qc_amd.core import TNTensor
    g, q = _qctn()
    cores = _cores(q, cplx)
    # one TNTensor core: the file stores tensor * scale
    first = q.cores[0]
    import torch
    T = torch.as_tensor
    q.cores_weights = {c: (TNTensor(T(cores[c] / 4.0), 4.0) if c == first else T(cores[c])) for c in q.cores}
    f = tmp_path / "cores.safetensors"
    q.save_cores(f, metadata={"step": 7})
    d = load_file(str(f))
    if cplx:
        assert set(d) == {f"core_{c}_{p}" for c in q.cores for p in ("real", "imag")}
        for c in q.cores:
            np.testing.assert_array_equal(d[f"core_{c}_real"], cores[c].real)
            np.testing.assert_array_equal(d[f"core_{c}_imag"], cores[c].imag)
    else:
        assert set(d) == {f"core_{c}" for c in q.cores}
        for c in q.cores:
            np.testing.assert_array_equal(d[f"core_{c}"], cores[c])
    # load: auto-scaled TNTensors, max|tensor| == 1, tensor * scale == saved value
    _, q2 = _qctn()
    meta = q2.load_cores(f)
    assert meta == {}  # the reference's load_file result is a dict, so its metadata is always {}
    for c in q.cores:
        t = q2.cores_weights[c]
        assert isinstance(t, TNTensor)
        assert np.isclose(float(t.tensor.abs().max()), 1.0)
        assert np.isclose(t.scale, np.abs(cores[c]).max())
        assert np.isclose(t.log_scale, np.log(np.abs(cores[c]).max()))
        np.testing.assert_allclose((t.tensor * t.scale).numpy(), cores[c], rtol=1e-15, atol=1e-15)


def test_safetensors_missing_keys_and_from_pretrained(tmp_path):
    from safetensors.numpy import save_file
    from tneq_qc_amd.core import QCTN
    g, q = _qctn()
    cores = _cores(q, False, 3)
    f = tmp_path / "partial.safetensors"
    keep = q.cores[1:]
    save_file({f"core_{c}": np.ascontiguousarray(cores[c]) for c in keep}, str(f))
    with pytest.raises(KeyError):
        q.load_cores(f)
    _, q3 = _qctn()
    before = {c: q3.cores_weights.get(c) for c in q3.cores}
    q3.load_cores(f, strict=False)
    assert q3.cores_weights.get(q3.cores[0]) is before[q3.cores[0]]
    for c in keep:
        np.testing.assert_allclose((q3.cores_weights[c].tensor * q3.cores_weights[c].scale).numpy(), cores[c])
    full = tmp_path / "full.safetensors"
    save_file({f"core_{c}": np.ascontiguousarray(cores[c]) for c in q.cores}, str(full))
    q4 = QCTN.from_pretrained(g, full, backend=_HostBackend())
    for c in q.cores:
        np.testing.assert_allclose((q4.cores_weights[c].tensor * q4.cores_weights[c].scale).numpy(), cores[c])


def test_save_without_backend_raises(tmp_path):
    from tneq_qc_amd.circuits import build_brick_wall_IM, incidence_to_graph
    from tneq_qc_amd.core import QCTN
    q = QCTN(incidence_to_graph(build_brick_wall_IM(3, 1)))
    q.backend = None
    with pytest.raises(RuntimeError):
        q.save_cores(tmp_path / "x.safetensors")
    with pytest.raises(RuntimeError):
        q.load_cores(tmp_path / "x.safetensors")


def _info(n, states=True, mx_nd=3, drop_state=None, drop_mx=None):
    ss = tuple(() if q == drop_state else (2,) for q in range(n)) if states else None
    ms = tuple(() if q == drop_mx else (4,) + (2,) * (mx_nd - 1) for q in range(n))
    return {"circuit_states_shapes": ss, "measure_shapes": ms, "measure_is_matrix": True}


def test_hip_tree_is_general_like_greedy():
    """GreedyStrategy.check_compatibility is always True (greedy_strategy.py:35-39); the HIP
    strategy replays its bookkeeping for open legs too, so it accepts every shape set and the
    'balanced' compiler picks it."""
    from tneq_qc_amd.contractor import HipTreeStrategy, StrategyCompiler
    _, q = _qctn(4, 2)
    s = HipTreeStrategy()
    n = q.nqubits
    for info in (_info(n, mx_nd=2), _info(n, mx_nd=4), _info(n, drop_mx=1), _info(n, drop_state=2),
                 _info(n, states=False)):
        assert s.check_compatibility(q, info)
    fn, name, cost = StrategyCompiler("balanced").compile(q, _info(n, drop_mx=0), backend=None)
    assert name == "hip_tree" and callable(fn)
