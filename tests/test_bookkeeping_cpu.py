"""Product host bookkeeping (tneq_qc_amd.core / contractor) == oracle restatement, bit-exact.

Index bookkeeping must be identical to the reference rules: core order,
edge lists, core axis layout, every einsum equation string, split/merge graph strings."""
import numpy as np
import pytest

from oracle import qctn_ref as R
from tneq_qc_amd.circuits import build_brick_wall_IM, incidence_to_graph
from tneq_qc_amd.contractor import EinsumStrategy as E
from tneq_qc_amd.core import QCTN


def random_graph(rng, nqubits, ncores):
    """Random graph in the reference's format (QCTNHelper.generate_random_example_graph idea,
    qctn.py:433-447): each qubit line visits a random subset of the cores in core order."""
    syms = [R.get_symbol(i) for i in range(ncores)]
    lines = []
    for _ in range(nqubits):
        chosen = [s for s in syms if rng.random() > 0.5] or [syms[int(rng.integers(ncores))]]
        line = f"-{int(rng.integers(2, 5))}-"
        for s in chosen:
            line += f"{s}-{int(rng.integers(2, 5))}-"
        lines.append(line)
    return "\n".join(lines)


def graphs():
    rng = np.random.default_rng(0)
    out = [incidence_to_graph(build_brick_wall_IM(n, c)) for n, c in ((2, 1), (4, 2), (8, 5), (10, 4), (13, 3))]
    out += [random_graph(rng, int(rng.integers(2, 7)), int(rng.integers(2, 9))) for _ in range(25)]
    # many cores -> symbols beyond the 52 ASCII letters
    out.append(incidence_to_graph(build_brick_wall_IM(30, 4)))
    return out


@pytest.mark.parametrize("g", graphs())
def test_adjacency_and_equations_match_oracle(g):
    p, o = QCTN(g), R.QCTNRef(g)
    assert p.cores == o.cores
    assert p.adjacency_table == o.adjacency_table
    assert [p.core_shape(c) for c in p.cores] == o.core_shapes()
    assert E.build_core_only_expression(p) == R.build_core_only_expression(o)
    n_in = sum(len(s) for s in o.circuit_inputs)
    assert E.build_with_vector_inputs_expression(p, [(2,)] * n_in)[0] == \
        R.build_with_vector_inputs_expression(o, [(2,)] * n_in)[0]
    assert E.build_with_inputs_expression(p, (2,) * n_in)[0] == R.build_with_inputs_expression(o, (2,) * n_in)[0]
    assert E.build_with_qctn_expression(p, QCTN(g))[0] == R.build_with_qctn_expression(o, R.QCTNRef(g))[0]


def test_workload_generators_match_oracle():
    for n, c in ((8, 5), (53, 10), (5, 1)):
        IM = build_brick_wall_IM(n, c)
        assert np.array_equal(IM, R.build_brick_wall_IM(n, c))
        assert incidence_to_graph(IM) == R.incidence_to_graph(IM)
    IM = build_brick_wall_IM(8, 5)
    IM[:, [2, 3, 5]] = 0
    assert incidence_to_graph(IM) == R.incidence_to_graph(IM)
    with pytest.raises(ValueError):
        incidence_to_graph(np.zeros((2, 2), int))


def test_self_expression_quirk_swaps_last_two_measurements():
    """einsum_strategy.py:517-519: the last two middle blocks are swapped."""
    g = incidence_to_graph(build_brick_wall_IM(3, 1))
    q = QCTN(g)
    eq, shapes = E.build_with_self_expression(q, ((2,),) * 3, ((4, 2, 2),) * 3, True)
    parts = eq.split("->")[0].split(",")
    mids = [p for p in parts if len(p) == 3 and p[0] == eq.split("->")[1]]
    assert len(mids) == 3
    # output symbols in core order are o0, o1, o2; blocks carry them in order o0, o2, o1
    outs = [s for s in E.build_with_vector_inputs_expression(q, [(2,)] * 3)[0].split("->")[1]]
    assert [m[1] for m in mids] == [outs[0], outs[2], outs[1]]
    assert len(shapes) == len(parts)


@pytest.mark.parametrize("n,c", [(4, 3), (6, 2), (8, 5)])
def test_split_and_merge_match_oracle(n, c):
    g = incidence_to_graph(build_brick_wall_IM(n, c))
    p, o = QCTN(g), R.QCTNRef(g)
    p1, p2 = p.split()
    g1, g2 = R.split_graph(o)
    assert (p1.graph, p2.graph) == (g1, g2)
    m = QCTN.merge(p1, p2)
    gm, _, _ = R.merge_graphs(R.QCTNRef(g1), R.QCTNRef(g2))
    assert m.graph == gm
    with pytest.raises(ValueError):
        p.split(0)


def test_split_rejects_interleaved_groups():
    q = QCTN("-2-a-2-b-2-c-2-\n-2-c-2-a-2-")
    with pytest.raises(ValueError, match="interleaved"):
        q.split(2)


def test_set_cores_validation():
    q = QCTN(incidence_to_graph(build_brick_wall_IM(3, 1)))
    z = np.zeros((2, 2, 2, 2))
    q.set_cores([z, z])
    assert q.cores_weights["a"].shape == (2, 2, 2, 2)
    with pytest.raises(ValueError):
        q.set_cores([z])
    with pytest.raises(ValueError):
        q.set_cores({"a": np.zeros(15), "b": z})
    with pytest.raises(TypeError):
        q.set_cores(z)
