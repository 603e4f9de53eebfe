"""Parity of the HIP contraction path (native plan: APPLY / permute / MFMA GEMM, slicing,
hoisting) against the oracle's exact numpy pairwise executor on identical inputs.

Tolerances (relative to max |reference|): complex128 1e-12, complex64 2e-5 — the fp64 / fp32
bounds of north_star ("amplitudes match ... to a stated fp64 tolerance").
"""
import numpy as np
import pytest

from oracle.contract_ref import contract as ref_contract

pytestmark = pytest.mark.gpu

TOL = {"complex128": 1e-12, "complex64": 2e-5, "float64": 1e-12, "float32": 2e-5}


def _err(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(1e-300, np.abs(b).max()))


def _run(task_or_eq, operands, dtype, dev, **kw):
    import torch
    from tneq_qc_amd.expression import HipContractExpression
    eq, shapes = task_or_eq
    e = HipContractExpression(eq, *shapes, **kw)
    ts = [torch.from_numpy(np.ascontiguousarray(o)).to(dev, getattr(torch, dtype)) for o in operands]
    return e, e(*ts).cpu().numpy()


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_c1_single_amplitude(dev, dtype):
    from tneq_qc_amd.circuits import config_task
    t = config_task("C1")
    ref = ref_contract(t.eq, *t.operands)
    _, out = _run((t.eq, t.shapes), t.operands, dtype, dev, optimize=t.path)
    assert _err(out, ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_full_state_vector_unitarity(dev, dtype):
    """10q depth-8, all outputs open: psi matches the oracle and sum |psi|^2 == 1 (KAT 1)."""
    from tneq_qc_amd.circuits import BrickWall, amplitude_task
    t = amplitude_task(BrickWall(10, 8, 3), list(range(10)))
    ref = ref_contract(t.eq, *t.operands)
    for opt in (t.path, "greedy"):
        _, out = _run((t.eq, t.shapes), t.operands, dtype, dev, optimize=opt)
        assert out.shape == (2,) * 10
        assert _err(out, ref) < TOL[dtype]
        assert abs((np.abs(out) ** 2).sum() - 1.0) < (1e-12 if dtype == "complex128" else 1e-5)


@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_cut_sliced_batch(dev, dtype):
    """Cut tree + index slicing (+ slice-invariant hoisting) == oracle; partial slice ranges sum."""
    import torch
    from tneq_qc_amd.circuits import BrickWall, amplitude_task
    t = amplitude_task(BrickWall(14, 8, 5), list(range(4, 10)), cut=7, n_slice=3)
    assert len(t.sliced) == 3
    ref = ref_contract(t.eq, *t.operands)
    e, out = _run((t.eq, t.shapes), t.operands, dtype, dev, optimize=t.path, slices=t.sliced)
    assert e.n_slices == 8
    assert _err(out, ref) < TOL[dtype]
    # ranks 0..3 of a 4-way shard, accumulated into one buffer == the full sum
    ts = [torch.from_numpy(np.ascontiguousarray(o)).to(dev, getattr(torch, dtype)) for o in t.operands]
    acc = torch.zeros(e.out_shape, dtype=getattr(torch, dtype), device=dev)
    for r in range(4):
        e(*ts, out=acc, slice_range=(r, 8, 4), accumulate=True)
    assert _err(acc.cpu().numpy(), ref) < TOL[dtype]


def test_core_only_ansatz_split_merge(dev):
    """C5 shape: the symmetry-breaking ansatz core-only contraction (einsum_strategy.py:136-194),
    complex128, via greedy and via the split/merge partition (qctn.py:1296-1506)."""
    from tneq_qc_amd.circuits import ansatz_qctn
    from tneq_qc_amd.contractor import EinsumStrategy
    from tneq_qc_amd.einsum import parse_equation, partition_path
    bw = ansatz_qctn()
    q = bw.qctn
    eq, shapes = EinsumStrategy.build_core_only_expression(q)
    ops = [bw.cores[c] for c in q.cores]
    ref = ref_contract(eq, *ops)
    assert ref.shape == (2,) * 16
    _, out = _run((eq, shapes), ops, "complex128", dev, optimize="greedy")
    assert _err(out, ref) < 1e-12
    half = q.ncores // 2
    path = partition_path(parse_equation(eq, shapes), [list(range(half)), list(range(half, q.ncores))])
    e, out2 = _run((eq, shapes), ops, "complex128", dev, optimize=path)
    assert _err(out2, ref) < 1e-12
    # the unitary circuit's core-only tensor is a 256 x 256 unitary (in legs x out legs)
    d = q.ncores  # noqa: F841


@pytest.mark.parametrize("dtype", ["float32", "float64", "complex64", "complex128"])
def test_random_networks_with_batch_modes(dev, dtype):
    """Random einsums incl. hyperedges (batch modes in 3+ operands and the output)."""
    rng = np.random.default_rng(11)
    letters = "abcdefghijklmnopq"
    for trial in range(12):
        nt = int(rng.integers(2, 6))
        ext = {c: int(rng.integers(1, 4)) for c in letters[:10]}
        terms = ["".join(rng.choice(list(letters[:10]), size=int(rng.integers(1, 5)), replace=False))
                 for _ in range(nt)]
        allc = sorted(set("".join(terms)))
        out = "".join(c for c in allc if rng.random() < 0.35)
        eq = ",".join(terms) + "->" + out
        ops = []
        for tm in terms:
            x = rng.standard_normal([ext[c] for c in tm])
            if dtype.startswith("complex"):
                x = x + 1j * rng.standard_normal(x.shape)
            ops.append(x.astype(dtype))
        ref = ref_contract(eq, *ops)
        _, got = _run((eq, [o.shape for o in ops]), ops, dtype, dev, optimize="greedy")
        assert got.shape == ref.shape, eq
        assert _err(got, ref) < TOL[dtype], (eq, trial)


def test_autograd_matches_torch(dev):
    """Gradients of a HIP expression (conj-other-operands rule) vs torch.einsum autograd."""
    import torch
    from tneq_qc_amd.expression import HipContractExpression
    rng = np.random.default_rng(2)
    a = rng.standard_normal((2, 3, 4)) + 1j * rng.standard_normal((2, 3, 4))
    b = rng.standard_normal((4, 5)) + 1j * rng.standard_normal((4, 5))
    c = rng.standard_normal((5, 2)) + 1j * rng.standard_normal((5, 2))
    eq = "ijk,kl,lm->ijm"
    e = HipContractExpression(eq, a.shape, b.shape, c.shape)
    tg = [torch.tensor(x, dtype=torch.complex128, device=dev, requires_grad=True) for x in (a, b, c)]
    tc = [torch.tensor(x, dtype=torch.complex128, requires_grad=True) for x in (a, b, c)]
    out = e(*tg)
    (out.abs() ** 2).sum().backward()
    ref = torch.einsum(eq, *tc)
    (ref.abs() ** 2).sum().backward()
    for g, r in zip(tg, tc):
        assert _err(g.grad.cpu().numpy(), r.grad.numpy()) < 1e-12


def test_graph_replay_matches_eager_and_rebuilds_on_new_pointers(dev):
    """The plan's hipGraph (captured launch sequence) is replayed while pointers / slice range are
    unchanged and rebuilt when they change; results equal the eager launch sequence bit for bit
    (same kernels, same order) and the oracle."""
    import torch
    from tneq_qc_amd.circuits import BrickWall, amplitude_task
    from tneq_qc_amd.expression import HipContractExpression
    t = amplitude_task(BrickWall(14, 8, 5), list(range(4, 10)), cut=7, n_slice=3)
    ref = ref_contract(t.eq, *t.operands)
    e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
    ts = [torch.from_numpy(np.ascontiguousarray(o)).to(dev, torch.complex64) for o in t.operands]
    out = torch.empty(e.out_shape, dtype=torch.complex64, device=dev)
    plan = e.plan(torch.complex64)
    e(*ts, out=out)
    b0 = plan.query("graph_builds")
    for _ in range(3):
        e(*ts, out=out)
    assert plan.query("graph_builds") == b0          # replayed, not re-captured
    g = out.clone()
    plan.profile(-1)                                  # profiling runs the eager launch sequence
    e(*ts, out=out)
    plan.profile(None)
    assert torch.equal(out, g)
    assert _err(g.cpu().numpy(), ref) < TOL["complex64"]
    ts2 = [x.clone() for x in ts]                     # new input pointers -> new graph
    out2 = e(*ts2)
    assert plan.query("graph_builds") == b0 + 1
    assert torch.equal(out2, g)
    part = e(*ts, slice_range=(1, e.n_slices, 2))     # new slice range -> new graph, partial sum
    assert plan.query("graph_builds") == b0 + 2
    part0 = e(*ts, slice_range=(0, e.n_slices, 2))
    assert _err((part + part0).cpu().numpy(), ref) < TOL["complex64"]


@pytest.mark.parametrize("dtype", ["complex64", "complex128", "float32", "float64"])
@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_fused_sweep_chains_random(dev, dtype, seed):
    """Random gate chains on a running tensor (binary and extent-3 legs, 1-2 contracted and
    1-2 new legs per gate, inner and outer positions): the plan fuses consecutive absorptions
    into SWEEP ops; the result equals the oracle's exact pairwise contraction."""
    import torch
    from tneq_qc_amd.expression import HipContractExpression
    rng = np.random.default_rng(100 + seed)
    syms = iter("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ")
    ext = {}
    cur = []
    for _ in range(rng.integers(8, 13)):
        s = next(syms)
        ext[s] = 3 if rng.random() < 0.15 else 2
        cur.append(s)
    terms = ["".join(cur)]
    for _ in range(rng.integers(6, 14)):
        kc = int(rng.integers(1, 3))
        pos = int(rng.integers(0, len(cur) - kc + 1))
        contracted = cur[pos:pos + kc] if rng.random() < 0.7 else list(rng.choice(cur, kc, replace=False))
        new = []
        for _ in range(int(rng.integers(1, 3))):
            s = next(syms)
            ext[s] = 2
            new.append(s)
        terms.append("".join(contracted) + "".join(new))
        cur = [c for c in cur if c not in contracted]
        cur[pos:pos] = new
    out = "".join(cur)
    eq = ",".join(terms) + "->" + out
    shapes = [tuple(ext[c] for c in t) for t in terms]
    cplx = dtype.startswith("complex")
    ops = []
    for shp in shapes:
        x = rng.standard_normal(shp)
        if cplx:
            x = x + 1j * rng.standard_normal(shp)
        ops.append(x / np.sqrt(np.prod(shp[-2:]) if len(shp) > 1 else 1))
    path = [(0, 1)] + [(len(terms) + i, i + 2) for i in range(len(terms) - 2)]
    ref = ref_contract(eq, *ops)
    e = HipContractExpression(eq, *shapes, optimize=path)
    plan = e.plan(getattr(torch, dtype))
    ts = [torch.from_numpy(np.ascontiguousarray(o)).to(dev, getattr(torch, dtype)) for o in ops]
    got = e(*ts).cpu().numpy()
    assert plan.query("n_sweep") >= 1, plan.describe()
    tol = {"complex64": 2e-5, "float32": 2e-5, "complex128": 1e-12, "float64": 1e-12}[dtype]
    assert _err(got, ref) < tol, plan.describe()
    # accumulate (beta = 1) into an existing output
    acc = torch.from_numpy(np.ascontiguousarray(ref)).to(dev, getattr(torch, dtype))
    e(*ts, out=acc, accumulate=True)
    assert _err(acc.cpu().numpy(), 2 * ref) < tol


@pytest.mark.parametrize("dtype", ["complex128", "complex64"])
def test_engine_contract_with_vector_inputs(dev, dtype):
    """Engine.contract_with_vector_inputs (engine.py:285-315), the reference's amplitude-vector
    API, on the 'hip' backend: psi of an 8-qubit brick wall on random product-state inputs
    == the oracle's vector-inputs equation (oracle.qctn_ref, einsum_strategy.py:258-318)
    contracted exactly; the expression is cached on the QCTN under the reference's attribute
    and reused; core-only / single-input / two-QCTN entry points too."""
    import torch
    from oracle import qctn_ref
    from tneq_qc_amd.backends import BackendFactory
    from tneq_qc_amd.circuits import BrickWall
    from tneq_qc_amd.core import Engine, QCTN
    bw = BrickWall(8, 4, 2)
    be = BackendFactory.create_backend("hip", device="cuda", dtype=dtype)
    q = QCTN(bw.graph, backend=be)
    q.set_cores({c: torch.from_numpy(bw.cores[c]) for c in q.cores})
    eng = Engine(backend=be)
    rng = np.random.default_rng(9)
    vecs = [(rng.standard_normal(2) + 1j * rng.standard_normal(2)) for _ in range(8)]
    psi = eng.contract_with_vector_inputs(q, vecs).cpu().numpy()
    qr = qctn_ref.QCTNRef(bw.graph)
    eq, _ = qctn_ref.build_with_vector_inputs_expression(qr, [(2,)] * 8)
    ref = ref_contract(eq, *vecs, *[bw.cores[c] for c in qr.cores])
    assert psi.shape == ref.shape and _err(psi, ref) < TOL[dtype]
    key = f"_contract_expr_vector_inputs_{tuple([torch.Size([2])] * 8)}"
    assert hasattr(q, key)
    expr = getattr(q, key)
    psi2 = eng.contract_with_vector_inputs(q, vecs).cpu().numpy()
    assert getattr(q, key) is expr and _err(psi2, ref) < TOL[dtype]
    # core-only (the 2^16-amplitude unitary of the 8 legs) and two-QCTN overlap
    u = eng.contract_core_only(q).cpu().numpy()
    eq_c, _ = qctn_ref.build_core_only_expression(qr)
    assert _err(u, ref_contract(eq_c, *[bw.cores[c] for c in qr.cores])) < TOL[dtype]
    ov = eng.contract_with_qctn(q, q).cpu().numpy()
    eq_q, _ = qctn_ref.build_with_qctn_expression(qr, qr)
    cores = [bw.cores[c] for c in qr.cores]
    assert _err(ov, ref_contract(eq_q, *cores, *cores)) < TOL[dtype]


def test_operand_binding_fast_path_tracks_changes(dev):
    """Repeated calls with the same operand objects take the bound fast path; an in-place update,
    an in-place transpose (strides), a replaced operand or a converted copy must all be seen."""
    import torch
    from tneq_qc_amd.circuits import BrickWall, amplitude_task
    from tneq_qc_amd.expression import HipContractExpression
    t = amplitude_task(BrickWall(10, 6, 11), list(range(3, 7)))
    e = HipContractExpression(t.eq, *t.shapes, optimize=t.path)
    ts = [torch.from_numpy(np.ascontiguousarray(o)).to(dev, torch.complex128) for o in t.operands]
    ops = [np.array(o, dtype=np.complex128) for o in t.operands]

    def check():
        out = e(*ts).cpu().numpy()
        assert _err(out, ref_contract(t.eq, *ops)) < 1e-12

    check()
    assert e._bound is not None and e._bound_call(tuple(ts)) is not None
    check()                                          # fast path, same result
    sq = next(i for i, o in enumerate(ops) if o.ndim == 4)
    ts[sq].mul_(0.5 + 0.25j)                          # in place: version bump
    ops[sq] = ops[sq] * (0.5 + 0.25j)
    check()
    ts[sq].transpose_(0, 1)                           # metadata: strides change
    ops[sq] = ops[sq].transpose(1, 0, 2, 3)
    check()
    k = next(i for i, o in enumerate(ops) if o.ndim == 4 and i != sq)
    ts[k] = ts[k] * 2                                 # a different object
    ops[k] = ops[k] * 2
    check()
    # operands the call converts (complex64 -> complex128) are not bound
    ts64 = [x.to(torch.complex64) for x in ts]
    e2 = HipContractExpression(t.eq, *t.shapes, optimize=t.path)
    e2(*[x.to(torch.complex128) if i else ts64[0] for i, x in enumerate(ts)])
    assert e2._bound is None
