"""The oracle pinned by hand-derived bookkeeping and semantic known-answer tests (CPU only).

The reference's own tests hold no golden values; these are the pins."""
import numpy as np
import pytest

from oracle.contract_ref import contract
from oracle.greedy_ref import greedy_contract
from oracle.qctn_ref import (QCTNRef, build_brick_wall_IM, build_core_only_expression,
                             build_with_inputs_expression, build_with_qctn_expression,
                             build_with_vector_inputs_expression, get_symbol, incidence_to_graph,
                             merge_graphs, random_cores, split_graph)

G3 = "-2-a-2-c-2-\n-2-a-2-b-2-\n-2-b-2-c-2-"


def test_get_symbol_rule():
    assert [get_symbol(i) for i in (0, 25, 26, 51)] == ["a", "z", "A", "Z"]
    assert get_symbol(52) == chr(192) and get_symbol(1000) == chr(1140)
    assert get_symbol(55296) == chr(55296 + 2048)  # surrogate block skipped


def test_hand_derived_adjacency_and_equations():
    """Derived by hand from qctn.py:591-722 and einsum_strategy.py:136-318 for G3."""
    q = QCTNRef(G3)
    assert q.cores == ["a", "b", "c"]
    a, b, c = q.adjacency_table
    assert [(e["neighbor_idx"], e["qubit_idx"]) for e in a["in_edge_list"]] == [(-1, 0), (-1, 1)]
    assert [(e["neighbor_idx"], e["qubit_idx"]) for e in a["out_edge_list"]] == [(2, 0), (1, 1)]
    assert [(e["neighbor_idx"], e["qubit_idx"]) for e in b["in_edge_list"]] == [(0, 1), (-1, 2)]
    assert [(e["neighbor_idx"], e["qubit_idx"]) for e in b["out_edge_list"]] == [(-1, 1), (2, 2)]
    assert [(e["neighbor_idx"], e["qubit_idx"]) for e in c["in_edge_list"]] == [(0, 0), (1, 2)]
    assert [(e["neighbor_idx"], e["qubit_idx"]) for e in c["out_edge_list"]] == [(-1, 0), (-1, 2)]
    assert build_core_only_expression(q)[0] == "abcd,defg,cghi->abefhi"
    assert build_with_vector_inputs_expression(q, [(2,)] * 3)[0] == "a,b,e,abcd,defg,cghi->fhi"
    assert build_with_inputs_expression(q, (2, 2, 2))[0] == "abe,abcd,defg,cghi->fhi"
    eq, _ = build_with_qctn_expression(q, QCTNRef(G3))
    # target reuses inputs a,b,e and outputs f,h,i; new internal symbols from j
    assert eq == "abcd,defg,cghi,abjk,kefl,jlhi->"


def test_core_order_follows_get_symbol_not_appearance():
    q = QCTNRef("-2-B-2-a-2-")
    assert q.cores == ["a", "B"]        # a (index 0) precedes B (index 27)


def test_incidence_and_brick_wall():
    IM = build_brick_wall_IM(4, 2)
    assert IM.shape == (4, 6)
    g = incidence_to_graph(IM)
    assert g.splitlines()[0] == "-2-a-2-d-2-"
    assert g.splitlines()[1] == "-2-a-2-c-2-d-2-f-2-"


def _unitary_task(n, cells, seed):
    g = incidence_to_graph(build_brick_wall_IM(n, cells))
    q = QCTNRef(g)
    return q, random_cores(q, seed)


def test_kat_unitarity_norm_one():
    q, cores = _unitary_task(6, 3, 1)
    eq, _ = build_with_vector_inputs_expression(q, [(2,)] * 6)
    zero = np.array([1.0, 0.0], complex)
    psi = contract(eq, *([zero] * 6), *[cores[c] for c in q.cores])
    assert abs((np.abs(psi) ** 2).sum() - 1) < 1e-12


def test_kat_identity_cores_product_state():
    q = QCTNRef(incidence_to_graph(build_brick_wall_IM(5, 2)))
    cores = random_cores(q, 0, kind="identity")
    rng = np.random.default_rng(3)
    vecs = [rng.standard_normal(2) + 1j * rng.standard_normal(2) for _ in range(5)]
    eq, _ = build_with_vector_inputs_expression(q, [(2,)] * 5)
    psi = contract(eq, *vecs, *[cores[c] for c in q.cores])
    # with identity cores every input flows to the output of the same qubit; the vectors are
    # consumed in core/in-edge order and outputs appear in core order
    in_q = [e["qubit_idx"] for t in q.adjacency_table for e in t["in_edge_list"] if e["neighbor_idx"] == -1]
    out_q = [e["qubit_idx"] for t in q.adjacency_table for e in t["out_edge_list"] if e["neighbor_idx"] == -1]
    by_q = {qq: vecs[k] for k, qq in enumerate(in_q)}
    expect = by_q[out_q[0]]
    for qq in out_q[1:]:
        expect = np.multiply.outer(expect, by_q[qq])
    assert np.allclose(psi, expect, atol=1e-13)


def test_kat_greedy_sandwich_projector_is_born_rule():
    q, cores = _unitary_task(4, 2, 5)
    zero = np.array([1.0, 0.0], complex)
    eq, _ = build_with_vector_inputs_expression(q, [(2,)] * 4)
    psi = contract(eq, *([zero] * 4), *[cores[c] for c in q.cores])
    out_q = [e["qubit_idx"] for t in q.adjacency_table for e in t["out_edge_list"] if e["neighbor_idx"] == -1]
    for x in ([0, 0, 0, 0], [1, 0, 1, 1], [0, 1, 1, 0]):
        mx = [np.outer(np.eye(2)[x[i]], np.eye(2)[x[i]])[None].astype(complex) for i in range(4)]
        r = greedy_contract(q, cores, [zero] * 4, mx)
        assert r.shape == (1,)
        assert abs(r[0] - abs(psi[tuple(x[qq] for qq in out_q)]) ** 2) < 1e-14


def test_kat_greedy_identity_measure_is_norm():
    q, cores = _unitary_task(4, 2, 6)
    zero = np.array([1.0, 0.0], complex)
    mx = [np.eye(2, dtype=complex)[None] for _ in range(4)]
    assert abs(greedy_contract(q, cores, [zero] * 4, mx)[0] - 1.0) < 1e-13


def test_kat_conditional_is_joint_over_marginal():
    """tests/test_probabilities.py:72-88 semantics through the (B, 2, K, K) stacking of
    engine_siamese.calculate_conditional_probability (engine_siamese.py:652-734)."""
    q, cores = _unitary_task(3, 2, 7)
    zero = np.array([1.0, 0.0], complex)
    P0 = np.array([[1, 0], [0, 0]], complex)
    I = np.eye(2, dtype=complex)
    mx = [np.stack([P0, I])[None], np.stack([P0, P0])[None], np.stack([I, I])[None]]  # target q0 | cond q1
    r = greedy_contract(q, cores, [zero] * 3, mx)
    joint = greedy_contract(q, cores, [zero] * 3, [P0[None], P0[None], I[None]])[0]
    marg = greedy_contract(q, cores, [zero] * 3, [I[None], P0[None], I[None]])[0]
    assert r.shape == (1, 2)
    assert abs(r[0, 0] - joint) < 1e-14 and abs(r[0, 1] - marg) < 1e-14
    assert abs(r[0, 0] / r[0, 1] - joint / marg) < 1e-12


def test_split_merge_contracts_to_the_same_tensor():
    """qctn.py:1296-1506: contracting the split halves over the boundary == unsplit (KAT 5)."""
    IM = build_brick_wall_IM(4, 3)
    q = QCTNRef(incidence_to_graph(IM))
    cores = random_cores(q, 9)
    g1, g2 = split_graph(q)
    q1, q2 = QCTNRef(g1), QCTNRef(g2)
    assert q1.cores == q.cores[: q.ncores // 2] and q2.cores == q.cores[q.ncores // 2:]
    full = contract(build_core_only_expression(q)[0], *[cores[c] for c in q.cores])
    t1 = contract(build_core_only_expression(q1)[0], *[cores[c] for c in q1.cores])
    t2 = contract(build_core_only_expression(q2)[0], *[cores[c] for c in q2.cores])
    # q1: per core order [inputs..., boundary outputs...]; reorder both to qubit order
    def qubit_axes(qq):
        ins, outs = [], []
        for t in qq.adjacency_table:
            for e in t["in_edge_list"]:
                if e["neighbor_idx"] == -1:
                    ins.append(("i", e["qubit_idx"]))
            for e in t["out_edge_list"]:
                if e["neighbor_idx"] == -1:
                    outs.append(("o", e["qubit_idx"]))
            # core-only output = each core's circuit in legs then out legs, core order
        order = []
        for t in qq.adjacency_table:
            order += [("i", e["qubit_idx"]) for e in t["in_edge_list"] if e["neighbor_idx"] == -1]
            order += [("o", e["qubit_idx"]) for e in t["out_edge_list"] if e["neighbor_idx"] == -1]
        return order
    a1, a2, af = qubit_axes(q1), qubit_axes(q2), qubit_axes(q)
    n = q.nqubits
    T1 = np.transpose(t1, [a1.index(("i", k)) for k in range(n)] + [a1.index(("o", k)) for k in range(n)])
    T2 = np.transpose(t2, [a2.index(("i", k)) for k in range(n)] + [a2.index(("o", k)) for k in range(n)])
    F = np.transpose(full, [af.index(("i", k)) for k in range(n)] + [af.index(("o", k)) for k in range(n)])
    d = 2 ** n
    assert np.allclose(T1.reshape(d, d) @ T2.reshape(d, d), F.reshape(d, d), atol=1e-12)
    # merge(split) reproduces the original graph (every line holds cores of both groups here)
    merged, _, _ = merge_graphs(q1, q2)
    assert merged == q.graph


def test_contract_pairwise_matches_numpy_einsum():
    rng = np.random.default_rng(0)
    for _ in range(20):
        a = rng.standard_normal((2, 3, 4)) + 1j * rng.standard_normal((2, 3, 4))
        b = rng.standard_normal((4, 3, 5))
        c = rng.standard_normal((5, 2))
        for eq in ("ijk,kjl,lm->im", "ijk,kjl,li->jl", "ijk,kjl,lm->mkij"):
            assert np.allclose(contract(eq, a, b, c), np.einsum(eq, a, b, c), atol=1e-12)
