"""The symbolic replay of GreedyStrategy's compute_fn (contractor/greedy_symbolic.py) vs the
oracle's literal restatement (oracle/greedy_ref.py, greedy_strategy.py:41-1080).

The replay emits one flat einsum; here it is evaluated by the oracle's numpy pairwise executor
(test infrastructure) on the same operands, and must equal the oracle's group-by-group result —
for the closed sandwich (2-, 3-, 4-D Mx), right_qctn=QCTN (the stale-neighbour quirk), no right
side, qubits without Mx or without a state (open legs), and dict containers.
"""
import numpy as np
import pytest


def _case(n, cells, seed):
    from oracle.qctn_ref import QCTNRef, random_cores
    from tneq_qc_amd.circuits import build_brick_wall_IM, incidence_to_graph
    from tneq_qc_amd.core import QCTN
    g = incidence_to_graph(build_brick_wall_IM(n, cells))
    return g, QCTN(g), QCTNRef(g), random_cores(QCTNRef(g), seed)


def _flat(q, cores, states, mx, right_qctn="symmetric", rcores=None):
    from tneq_qc_amd.contractor.greedy_symbolic import greedy_equation

    def present(c, k):
        if c is None:
            return False
        return k in c if isinstance(c, dict) else k < len(c)

    sd = {k: states[k].shape[0] for k in q.qubit_indices if present(states, k)}
    md = {k: (mx[k].ndim, mx[k].shape[-2], mx[k].shape[-1]) for k in q.qubit_indices
          if present(mx, k) and mx[k] is not None}
    cn = {c: cores[c].ndim for c in q.cores}
    rn = {c: rcores[c].ndim for c in rcores} if rcores is not None else None
    return greedy_equation(q, sd, md, cn, right_qctn, rn)


def _operands(recipe, cores, states, mx, rcores=None):
    ops = []
    for kind, key in recipe:
        if kind == "L":
            ops.append(cores[key])
        elif kind == "R":
            ops.append(np.conj(cores[key]))
        elif kind == "Rq":
            ops.append(rcores[key])
        elif kind == "S":
            ops.append(states[key])
        else:
            ops.append(mx[key])
    return ops


def _check(got_eq, recipe, ref, cores, states, mx, rcores=None):
    from oracle.contract_ref import contract
    got = contract(got_eq, *_operands(recipe, cores, states, mx, rcores))
    assert np.shape(got) == np.shape(ref)
    scale = max(np.abs(ref).max(), 1e-300)
    assert np.abs(got - ref).max() / scale < 1e-12


def _mx(rng, n, kind, B=3):
    if kind == 2:
        return [rng.standard_normal((2, 2)) + 1j * rng.standard_normal((2, 2)) for _ in range(n)]
    if kind == 3:
        return [rng.standard_normal((B, 2, 2)) + 1j * rng.standard_normal((B, 2, 2)) for _ in range(n)]
    return [rng.standard_normal((B, 2, 2, 2)) + 1j * rng.standard_normal((B, 2, 2, 2)) for _ in range(n)]


@pytest.mark.parametrize("n,cells,kind", [(3, 1, 3), (3, 2, 2), (4, 2, 3), (4, 2, 4), (5, 2, 3)])
def test_closed_sandwich(n, cells, kind):
    from oracle.greedy_ref import greedy_contract
    g, q, qr, cores = _case(n, cells, 100 + n)
    rng = np.random.default_rng(n)
    states = [rng.standard_normal(2) + 1j * rng.standard_normal(2) for _ in range(n)]
    mx = _mx(rng, n, kind)
    eq, rec = _flat(q, cores, states, mx)
    _check(eq, rec, greedy_contract(qr, cores, states, mx), cores, states, mx)


def test_right_qctn_quirk():
    from oracle.greedy_ref import greedy_contract
    from oracle.qctn_ref import QCTNRef, random_cores
    from tneq_qc_amd.core import QCTN
    g, q, qr, cores = _case(4, 2, 11)
    rcores = random_cores(QCTNRef(g), 12)
    rng = np.random.default_rng(4)
    states = [np.array([0.6, 0.8j], complex) for _ in range(4)]
    mx = _mx(rng, 4, 3)
    ref = greedy_contract(qr, cores, states, mx, right_qctn=QCTNRef(g), right_cores=rcores)
    eq, rec = _flat(q, cores, states, mx, right_qctn=QCTN(g), rcores=rcores)
    _check(eq, rec, ref, cores, states, mx, rcores)


def test_no_right_side_and_open_legs():
    from oracle.greedy_ref import greedy_contract
    g, q, qr, cores = _case(3, 2, 31)
    rng = np.random.default_rng(5)
    states = [rng.standard_normal(2) + 0j for _ in range(3)]
    mx = _mx(rng, 3, 3)
    # right_qctn=None: L and M only; the leftover Mx-side merged tensors carry more legs than
    # _contract_remaining writes subscripts for (:1030-1041), so the reference's torch.einsum
    # fails — the oracle (numpy) and the replay fail the same way
    with pytest.raises(ValueError):
        greedy_contract(qr, cores, states, mx, right_qctn=None)
    with pytest.raises(RuntimeError, match="number of subscripts"):
        _flat(q, cores, states, mx, right_qctn=None)
    # a qubit without Mx (dict container) and a qubit without a state
    mxd = {0: mx[0], 2: mx[2]}
    eq, rec = _flat(q, cores, states, mxd)
    _check(eq, rec, greedy_contract(qr, cores, states, mxd), cores, states, mxd)
    st2 = states[:2]
    eq, rec = _flat(q, cores, st2, mx)
    _check(eq, rec, greedy_contract(qr, cores, st2, mx), cores, st2, mx)


def test_equation_is_deterministic_and_uses_every_leaf_once_per_side():
    g, q, qr, cores = _case(4, 2, 3)
    states = [np.array([1.0, 0.0], complex)] * 4
    mx = [np.eye(2, dtype=complex)[None].repeat(2, 0)] * 4
    e1, r1 = _flat(q, cores, states, mx)
    e2, r2 = _flat(q, cores, states, mx)
    assert e1 == e2 and r1 == r2
    assert sorted(k for k, _ in r1 if k in ("L", "R")) == ["L"] * q.ncores + ["R"] * q.ncores
    assert sum(1 for k, _ in r1 if k == "M") == 4 and sum(1 for k, _ in r1 if k == "S") == 8
    assert e1.endswith("->a")
