"""Full-size parity on the GPU (BASELINE.json configs), against the oracle where it finishes in
seconds and through size-independent properties where it does not.

* C2 (30q depth-14, one amplitude): the whole network against the oracle.
* C3 / C4 / C3d / C4g: ONE SLICE of each configuration (the same network, path, cut and sliced
  legs as bench.py).  C4 / C3d: left/right sweeps, the slice-invariant boundary GEMM (K = 2^11 /
  2^8) and the deferred sweep tails absorbed after it per slice (einsum.partition_path
  defer=...).  C3 / C4g (the plain partition path): the boundary GEMM per slice at K = 2^10 /
  2^16, C4g's on producer-split f16 planes with split-K.  Against the oracle's exact numpy
  contraction
  of the same sliced operands (oracle.contract_ref.sliced_operands, the slice enumeration of
  tq_plan_execute).  Normwise bounds (relative to max|amp|): complex64 1e-5, complex128 1e-12.
  Componentwise (the Gauss-3M imaginary part): every amplitude with
  |amp| >= 1e-2 max|amp| within 1e-3 relative, the normwise bound carried down to it.
* C3 / C3d / C4 / C4g whole job EXACTLY as bench.py launches it (SlicedContraction at world 1
  over the full slice range: C4 8 slice lanes / C3 and C3d 32 / C4g 4, the f16-split boundary
  GEMM with operand-max words (C3 / C4g: lane-batched, per-lane words, lane_sum), lane-merged
  sweep launches, the captured hipGraph replayed)
  against the oracle's sum over all slices (oracle.contract_ref.contract_sliced; the partial sums
  the reference reduces at distributed_engine.py:1477-1497).
* Lane skew: slices whose operands are 2^36 per cut leg larger than slice 0's, but whose
  contribution is exactly zero, batched in the same lanes as slice 0: the result must be slice
  0's amplitudes at full complex64 accuracy (a scale shared across lanes would flush them).
* C3 / C4 / C3d / C4g whole job: sliced + hoisted execution equals the unsliced contraction (1e-5), every
  4-way rank shard of the slices sums to the full result, and 0 < sum |amp|^2 <= 1 (the
  amplitudes are a sub-block of a unitary circuit's |psi>).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# complex64: SURVEY.md §8(c)'s fp32 bound, 1e-5 of max|amp| (measured on the production launches,
# profiles/accuracy_r06.json: 0.8e-6 .. 2.6e-6 normwise, as the oracle's own numpy complex64 run
# of the same path: 0.9e-6 .. 1.2e-6); componentwise 100x that on |amp| >= 1e-2 max (measured
# <= 1.7e-4, numpy complex64 7.7e-5)
TOL = {"complex64": 1e-5, "complex128": 1e-12}


def _expr_and_ops(task, dev, dtype, sliced=True):
    import torch
    from tneq_qc_amd.expression import HipContractExpression
    e = HipContractExpression(task.eq, *task.shapes, optimize=task.path,
                              slices=task.sliced if sliced else ())
    ops = [torch.from_numpy(o).to(dev, dtype) for o in task.operands]
    return e, ops


def test_c2_single_amplitude_vs_oracle(dev):
    import torch
    from oracle.contract_ref import contract as ref_contract
    from tneq_qc_amd.circuits import config_task
    t = config_task("C2")
    ref = ref_contract(t.eq, *t.operands, path=t.path)
    for dt, tol in ((torch.complex128, TOL["complex128"]), (torch.complex64, TOL["complex64"])):
        e, ops = _expr_and_ops(t, dev, dt)
        got = e(*ops).cpu().numpy()
        assert abs(got - ref) / abs(ref) < tol


@pytest.mark.parametrize("cfg", ["C3", "C4"])
def test_chain_launch_equals_one_launch_per_level(dev, cfg):
    """Consecutive small hoisted sweep2 levels run as ONE chain launch by default (a workgroup
    per stream, one-chunk layouts, LDS hand-offs between the ops of a stream: tq_plan.cpp
    Plan::seq_once, S2Launch::seq) -- C3's and C4's first levels; the same plan with
    "sweep_chain" = 0 launches them level by level (multi-chunk layouts).  The per-element
    arithmetic is the same gate sequence, so the two agree to rounding; a replay is exact.
    (C2's levels with TQ_S2_SEQCH=4 are the same mechanism on one stream.)"""
    import torch
    from tneq_qc_amd.circuits import config_task
    t = config_task(cfg)
    for dt, tol in ((torch.complex128, 1e-13), (torch.complex64, 1e-6)):
        e, ops = _expr_and_ops(t, dev, dt)
        p = e.plan(dt)
        assert p.query("n_chain_launches") == 1
        a = e(*ops).cpu().numpy()
        p.set("sweep_chain", 0)
        assert p.query("n_chain_launches") == 0
        b = e(*ops).cpu().numpy()
        p.set("sweep_chain", 1)
        c = e(*ops).cpu().numpy()
        assert np.abs(a - b).max() <= tol * np.abs(b).max() and np.array_equal(a, c)


def test_cooperative_chain_equals_one_launch_per_level(dev):
    """C2's 26 levels of one multi-chunk sweep2 op run as ONE cooperative launch with
    "sweep_coop" = 1 (8 workgroups; complex128: 32 + 2 ops), each op's chunks spread over them, a counter barrier between the ops, sc1 loads /
    stores: tq_plan.cpp Plan::coop_once, S2Launch::sync); "sweep_coop" = 0 (the default, measured
    faster) launches them level by level.  Same descriptors, same arithmetic: the results are bit-identical, on every one of many
    graph replays (a missed barrier shows up as a stale chunk), eager and captured, and no wait
    gave up."""
    import torch
    from tneq_qc_amd.circuits import config_task
    t = config_task("C2")
    for dt in (torch.complex128, torch.complex64):
        e, ops = _expr_and_ops(t, dev, dt)
        p = e.plan(dt)
        p.set("sweep_coop", 1)
        assert p.query("n_coop_launches") >= 1 and p.query("n_coop_ops") >= 20   # c128: 32 + 2 ops
        p.set("sweep_coop", 0)
        ref = e(*ops).cpu().numpy()
        p.set("sweep_coop", 1)
        refd = torch.from_numpy(ref).to(dev)
        for graph in (1, 0):
            p.set("graph", graph)
            bad = sum(int(not torch.equal(e(*ops), refd)) for _ in range(40))
            assert bad == 0, (dt, graph, bad)
        p.set("graph", 1)
        assert p.query("coop_timeouts") == 0


_ORACLE_SLICES = {}


def _oracle_slice(cfg, sid):
    """Exact (complex128) amplitudes of slice `sid` of config `cfg`, cached per session."""
    key = (cfg, sid)
    if key not in _ORACLE_SLICES:
        from oracle.contract_ref import contract as ref_contract, sliced_operands
        from tneq_qc_amd.circuits import config_task
        t = config_task(cfg)
        eq, ops = sliced_operands(t.eq, t.operands, t.sliced, sid)
        _ORACLE_SLICES[key] = ref_contract(eq, *ops, path=t.path)
    return _ORACLE_SLICES[key]


@pytest.mark.parametrize("cfg,sid", [("C4", 0), ("C4", 5), ("C3", 0), ("C3", 37), ("C4g", 5),
                                     ("C3d", 37)])
@pytest.mark.parametrize("dtype", ["complex64", "complex128"])
def test_bench_config_slice_vs_oracle(dev, cfg, sid, dtype):
    import torch
    from tneq_qc_amd.circuits import config_task
    t = config_task(cfg)
    e, ops = _expr_and_ops(t, dev, getattr(torch, dtype))
    got = e(*ops, slice_range=(sid, sid + 1, 1)).cpu().numpy()
    ref = _oracle_slice(cfg, sid)
    assert got.shape == ref.shape
    amax = np.abs(ref).max()
    err = np.abs(got - ref)
    rel = err.max() / amax
    assert rel < TOL[dtype], (cfg, sid, dtype, rel)
    big = np.abs(ref) >= 1e-2 * amax
    comp = (err[big] / np.abs(ref[big])).max()
    assert comp < TOL[dtype] * 100, (cfg, sid, dtype, comp)


_ORACLE_FULL = {}


def _oracle_full(cfg):
    """Exact (complex128) sum over every slice of config `cfg`, cached per session.  C3d / C4g are
    the same networks as C3 / C4 (same equation and operands, another path): the sum over all
    slices is the full amplitude block either way, so they share C3's / C4's oracle."""
    cfg = {"C3d": "C3", "C4g": "C4"}.get(cfg, cfg)
    if cfg not in _ORACLE_FULL:
        from oracle.contract_ref import contract_sliced
        from tneq_qc_amd.circuits import config_task
        t = config_task(cfg)
        _ORACLE_FULL[cfg] = contract_sliced(t.eq, t.operands, t.sliced, t.path)
    return _ORACLE_FULL[cfg]


def _check(got, ref, tol, what):
    amax = np.abs(ref).max()
    err = np.abs(got - ref)
    rel = err.max() / amax
    assert rel < tol, (what, rel)
    big = np.abs(ref) >= 1e-2 * amax
    comp = (err[big] / np.abs(ref[big])).max()
    assert comp < tol * 100, (what, comp)


def _production_plan_checks(e, cfg, lanes):
    import torch
    plan = e.plan(torch.complex64)
    assert plan.query("lanes") == lanes, plan.query("lanes")
    d = plan.describe()
    gemm = [l for l in d.splitlines() if " GEMM " in l]
    assert len(gemm) == 1 and "amax<-" in gemm[0], gemm
    if cfg in ("C3d", "C4"):
        # deferred tails: the boundary GEMM is slice-invariant (run once, fed by its producers'
        # max words); the slices run only the absorbed tails, lane-merged
        assert gemm[0].startswith("[once]"), gemm
        return
    # the lane-batched boundary GEMM fed by its producers' max words, summed over lanes
    assert " lanes" in d and "lane-sum" in d, d
    if cfg == "C4g":
        # both halves' per-slice expanding chains as dense ops of one level (tin 16 and 8: one
        # mixed sweepd launch, tq_sweepd.hip)
        dense = [l for l in d.splitlines() if "SWEEP2 DENSE" in l]
        assert any("tin=16" in l for l in dense) and any("tin=8" in l for l in dense), dense
        # the boundary GEMM on operands pre-split by those dense ops (tq_gemmp.hip)
        assert plan.query("planes_gemm") == 1, d
        assert any("planes(A)" in l for l in dense) and any("planes(B)" in l for l in dense), dense


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg,lanes", [("C3", 32), ("C3d", 32), ("C4", 8), ("C4g", 4)])
def test_bench_launch_vs_oracle(dev, cfg, lanes):
    import torch
    from tneq_qc_amd.circuits import config_task
    from tneq_qc_amd.distributed import SlicedContraction
    t = config_task(cfg)
    e, ops = _expr_and_ops(t, dev, torch.complex64)
    _production_plan_checks(e, cfg, lanes)
    job = SlicedContraction(e)
    out = torch.empty(e.out_shape, dtype=torch.complex64, device=dev)
    plan = e.plan(torch.complex64)
    g0 = plan.query("graph_launches")
    res = []
    for _ in range(3):   # first call captures the graph, the next ones replay it (as bench.py)
        job(*ops, out=out)
        res.append(out.cpu().numpy().copy())
    assert plan.query("graph_launches") >= g0 + 2
    ref = _oracle_full(cfg)
    assert res[0].shape == ref.shape
    for r in res:
        _check(r, ref, TOL["complex64"], cfg)
    assert np.array_equal(res[1], res[2])   # replays are deterministic


@pytest.mark.timeout(900)
def test_planes_gemm_equals_split_kernel(dev):
    """C4g's boundary GEMM on producer-split operands (the dense ops store six f16 term planes
    scaled from a bound of their output; tq_gemmp.hip: Gauss 3M x 3 term products from LDS-DMA
    staged planes, split-K partials, one combine pass summing the lanes) against the same plan on
    the GEMM-side split kernel ("gemm_planes" = 0) and both against the oracle's sum over all
    slices.  The two kernels round differently (the planes' scale comes from a bound, not the
    true max), so they agree to the complex64 tolerance, not bitwise."""
    import torch
    from tneq_qc_amd.circuits import config_task
    t = config_task("C4g")
    e, ops = _expr_and_ops(t, dev, torch.complex64)
    plan = e.plan(torch.complex64)
    assert plan.query("planes_gemm") == 1
    on = e(*ops).cpu().numpy()
    assert plan.query("planes_active") == 1 and plan.query("planes_bytes") > 0
    plan.set("gemm_planes", 0)
    off = e(*ops).cpu().numpy()
    plan.set("gemm_planes", 1)
    again = e(*ops).cpu().numpy()
    ref = _oracle_full("C4g")
    _check(on, ref, TOL["complex64"], "planes")
    _check(off, ref, TOL["complex64"], "split")
    assert np.abs(on - off).max() / np.abs(ref).max() < 2 * TOL["complex64"]   # two complex64 results
    assert np.array_equal(on, again)
    # partial lane batches (3 + 5 slices over 4-lane batches): a launch of fewer entries than lanes
    # may take more split-K partials than a full one (planes_gemm_workspace covers every size)
    p1 = e(*ops, slice_range=(0, 3, 1)).cpu().numpy()
    p2 = e(*ops, slice_range=(3, e.n_slices, 1)).cpu().numpy()
    assert np.abs(p1 + p2 - on).max() / np.abs(ref).max() < 2 * TOL["complex64"]


@pytest.mark.parametrize("cfg,lanes", [("C3", 32), ("C4", 8), ("C3d", 32), ("C4g", 4)])
def test_lane_skew_per_lane_scales(dev, cfg, lanes):
    import torch
    from tneq_qc_amd.circuits import config_task
    t = config_task(cfg)
    terms = t.eq.split("->")[0].split(",")
    opsn = [o.copy() for o in t.operands]
    n_var = int(np.log2(lanes))   # the last legs vary inside slice 0's lane batch
    for q, s in enumerate(t.sliced):
        holders = [i for i, x in enumerate(terms) if s in x]
        assert len(holders) == 2, (s, holders)   # a cut bond: one core on each side
        zi, bi = holders
        ax_z, ax_b = terms[zi].index(s), terms[bi].index(s)
        idx = [slice(None)] * opsn[zi].ndim
        idx[ax_z] = slice(1, None)
        opsn[zi][tuple(idx)] = 0            # every slice with this leg at 1 contributes 0 ...
        if q < len(t.sliced) - n_var:
            continue
        idx = [slice(None)] * opsn[bi].ndim
        idx[ax_b] = slice(1, None)
        opsn[bi][tuple(idx)] *= 2.0 ** 36   # ... but its other operand is 2^36 larger
    from tneq_qc_amd.expression import HipContractExpression
    e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
    _production_plan_checks(e, cfg, lanes)
    ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in opsn]
    got = e(*ops).cpu().numpy()
    assert np.isfinite(got).all()
    _check(got, _oracle_slice(cfg, 0), TOL["complex64"], cfg)


@pytest.mark.parametrize("cfg", ["C3", "C4", "C3d", "C4g"])
def test_sliced_equals_unsliced(dev, cfg):
    import torch
    from tneq_qc_amd.circuits import config_task
    t = config_task(cfg)
    e, ops = _expr_and_ops(t, dev, torch.complex64)
    sliced = e(*ops)
    e0, _ = _expr_and_ops(t, dev, torch.complex64, sliced=False)
    full = e0(*ops)
    # two complex64 results, each within TOL of the exact amplitudes (checked against the oracle
    # above): their difference is bounded by 2 TOL (C4g's unsliced path runs ONE K = 2^19 GEMM)
    err = (sliced - full).abs().max().item() / full.abs().max().item()
    assert err < 2 * TOL["complex64"], err
    # 4-way shard of the slices accumulated == full sum
    acc = torch.zeros_like(full)
    for r in range(4):
        e(*ops, out=acc, slice_range=(r, e.n_slices, 4), accumulate=True)
    err2 = (acc - full).abs().max().item() / full.abs().max().item()
    assert err2 < 2 * TOL["complex64"], err2
    p = (full.abs() ** 2).sum().item()
    assert 0.0 < p <= 1.0 + 1e-4


def test_c4x4_holds_the_c4_block(dev):
    """C4x4 (bench secondary line): the C4 network with qubits 16 and 37 open too, C4's fixed bits
    elsewhere -- one contraction of 4 blocks.  Its (q16, q37) = C4's-bits sub-block must be C4's
    amplitudes (C4 itself is checked against the oracle above), and 0 < sum |amp|^2 <= 1."""
    import torch
    from tneq_qc_amd.circuits import config_task
    t4, t = config_task("C4x4"), config_task("C4")
    e4, ops4 = _expr_and_ops(t4, dev, torch.complex64)
    e, ops = _expr_and_ops(t, dev, torch.complex64)
    big = e4(*ops4).cpu().numpy()
    ref = e(*ops).cpu().numpy()
    idx = tuple(t.fixed_bits[q] if q in (16, 37) else slice(None) for q in t4.open_qubits)
    assert [q for q in t4.open_qubits if q not in (16, 37)] == t.open_qubits
    sub = big[idx]
    assert sub.shape == ref.shape
    assert np.abs(sub - ref).max() / np.abs(ref).max() < 2 * TOL["complex64"]   # two complex64 results
    p = float((np.abs(big) ** 2).sum())
    assert 0.0 < p <= 1.0 + 1e-4
