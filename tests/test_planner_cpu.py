"""Host planner + native plan compiler on the CPU (no GPU needed: tq_plan_create only compiles;
device memory is taken at the first execute).  Also checks the C ABI exports."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

import tneq_qc_amd
from tneq_qc_amd import _lib
from tneq_qc_amd.circuits import BrickWall, amplitude_task, config_task
from tneq_qc_amd.einsum import (choose_slices, greedy_path, linear_path, parse_equation,
                                partition_path, path_info, validate_path)

ROOT = Path(__file__).resolve().parents[1]


def test_library_exports_every_header_symbol():
    header = (ROOT / "include" / "tneqhip.h").read_text()
    declared = set(re.findall(r"\b(tq_[a-z_]+)\s*\(", header))
    L = _lib.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert declared == set(_lib.EXPORTED)
    assert L.tq_version() >= 1


def test_parse_equation_errors():
    with pytest.raises(ValueError):
        parse_equation("ab,bc->ac", [(2, 3)])
    with pytest.raises(ValueError):
        parse_equation("ab,bc->ac", [(2, 3), (4, 2)])
    with pytest.raises(ValueError):
        parse_equation("aa->a", [(2, 2)])
    with pytest.raises(ValueError):
        parse_equation("ab->c", [(2, 2)])
    n = parse_equation("ab,bc", [(2, 3), (3, 4)])   # implicit output = 'ac'
    assert [n.symbols[m] for m in n.out] == ["a", "c"]


@pytest.mark.parametrize("cfg", ["C1", "C2"])
def test_paths_valid_and_sweep_is_narrow(cfg):
    t = config_task(cfg)
    net = t.network()
    validate_path(len(net.terms), t.path)
    info = path_info(net, t.path)
    d = t.circuit.depth
    assert info.max_size <= 2 ** (d + 2)          # a line sweep keeps ~2^d legs
    g = greedy_path(net)
    validate_path(len(net.terms), g)
    lp, root = linear_path(net)
    validate_path(len(net.terms), lp)


def test_partition_and_slicing_choose_cut_legs():
    t = amplitude_task(BrickWall(14, 8, 1), list(range(4, 10)), cut=7, n_slice=2)
    net = t.network()
    sl = [net.symbols.index(s) for s in t.sliced]
    assert not set(sl) & set(net.out)
    info0 = path_info(net, t.path)
    info = path_info(net, t.path, sl)
    assert info.n_slices == 4
    assert info.slice_flops < info0.flops


def _plan(task, dtype="complex64"):
    import torch
    from tneq_qc_amd.expression import HipContractExpression
    e = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
    return e, e.plan(getattr(torch, dtype))


def test_native_plan_lowering_c1_is_all_apply():
    """C1's sweep lowers to streaming passes only (APPLY, or fused SWEEP chains of APPLY steps):
    no permute, no GEMM; every one of the 71 pairwise steps is covered by exactly one op."""
    e, p = _plan(config_task("C1"))
    assert p.query("n_apply") + p.query("n_sweep") == p.query("n_kernels")
    assert p.query("n_permute") == 0 and p.query("n_gemm") == 0
    assert p.query("n_apply") + p.query("n_sweep_gates") == len(e.path)
    assert p.query("n_sweep") > 0
    assert p.n_slices == 1


def test_native_plan_c4_structure():
    e, p = _plan(config_task("C4g"))
    assert p.n_slices == 8
    assert p.query("n_gemm") == 1                        # the boundary GEMM
    d = p.describe().splitlines()
    gemm = [l for l in d if "GEMM" in l]
    assert "M=1024 N=1024" in gemm[0] and "[slice]" in gemm[0]
    assert p.query("n_ops_once") > 0.5 * p.query("n_kernels")   # most of the sweep is hoisted
    # left / right sweeps are the two independent branches, the GEMM is the join
    assert any(" b0 " in l for l in d) and any(" b1 " in l for l in d)
    assert " b2 " in gemm[0]
    assert p.query("flops") == pytest.approx(p.query("flops_once") + 8 * p.query("flops_slice"), rel=1e-6)


def test_c4_gemm_operand_max_comes_from_its_producers():
    """The C4 boundary GEMM (complex64, K-outer fast path) reads both operands' max |x| from the
    per-slice sweep ops that store them (csrc/tq_plan.cpp assign_amax), not from a pre-pass."""
    import re
    e, p = _plan(config_task("C4g"))
    d = p.describe().splitlines()
    ops = [l for l in d if l.startswith("[once]") or l.startswith("[slice]")]
    gemm = [l for l in ops if "GEMM" in l]
    m = re.search(r"amax<-op(\d+),op(\d+)", gemm[0])
    assert m, gemm[0]
    for j in (int(m.group(1)), int(m.group(2))):
        assert "SWEEP2" in ops[j] and ops[j].startswith("[slice]")
        assert ops.index(gemm[0]) > j


def _schedule(d):
    once, per = [], []
    for l in d:
        if l.startswith("# once"):
            once.append([int(x) for x in l.split()[2:]])
        elif l.startswith("# slice"):
            per.append([int(x) for x in l.split()[2:]])
    return once, per


def test_launch_schedule_covers_every_op_once_and_batches_sweeps():
    """Every op appears in exactly one launch of its set (hoisted / per slice), launches with more
    than one op hold only independent SWEEP2 ops, and the C4g sweeps share launches."""
    e, p = _plan(config_task("C4g"))
    d = p.describe().splitlines()
    ops = [l for l in d if l.startswith("[once]") or l.startswith("[slice]")]
    once, per = _schedule(d)
    seen = sorted(j for g in once + per for j in g)
    assert seen == list(range(len(ops)))
    for g in once:
        assert all(ops[j].startswith("[once]") for j in g)
    for g in per:
        assert all(ops[j].startswith("[slice]") for j in g)
    for g in once + per:
        if len(g) > 1:
            assert len(g) <= 32 and all("SWEEP2" in ops[j] for j in g)
    # chain launches merge runs of hoisted levels (each run: one launch)
    chains = [l for l in d if l.startswith("# chain launch")]
    merged = sum(int(l.split("..")[1].split(",")[0]) - int(l.split("entries ")[1].split("..")[0]) for l in chains)
    assert p.query("n_launch_once") == len(once) - merged and p.query("n_launch_slice") == len(per)
    assert p.query("n_sweep2") > 60 and len(once) < p.query("n_ops_once")
    # the GEMM of a slice waits for both branch sweeps: it is alone in its launch, after them
    gi = [k for k, g in enumerate(per) for j in g if "GEMM" in ops[j]]
    assert len(gi) == 1 and len(per[gi[0]]) == 1 and gi[0] > 0


def test_sweep_tiles_keep_32_columns_on_large_tensors():
    """Tiles with more than 2^(13-5) positions (fewer than 32 columns per chunk) are reserved for
    tensors of at most 2^22 elements (SWEEP2 layout rule, csrc/tq_plan.cpp s2_layout)."""
    import re
    e, p = _plan(config_task("C4g"))
    n_wide = 0
    for l in p.describe().splitlines():
        m = re.search(r"SWEEP2 gates=(\d+) tin=(\d+) tout=(\d+) cols=(\d+) C=(\d+)", l)
        if not m:
            continue
        g, tin, tout, cols, C = map(int, m.groups())
        assert 1 <= g <= 16
        if max(tin, tout) > 256:
            n_wide += 1
            assert max(tin, tout) * cols <= 1 << 22
        elif max(tin, tout) * cols > 1 << 22:
            assert C >= 32 or cols < 32
    assert n_wide > 0


def test_plan_rejects_bad_paths():
    from tneq_qc_amd.expression import HipContractExpression
    with pytest.raises(ValueError):
        HipContractExpression("ab,bc,cd->ad", (2, 2), (2, 2), (2, 2), optimize=[(0, 1), (0, 2)])
    with pytest.raises(ValueError):
        HipContractExpression("ab,bc->ac", (2, 2), (2, 2), slices=["a"])


def test_plan_create_errors_map_to_valueerror():
    import torch
    from tneq_qc_amd.expression import NativePlan
    from tneq_qc_amd.einsum import Network
    net = Network([[0, 1], [1, 2]], [0, 2], {0: 2, 1: 3, 2: 2})
    with pytest.raises(ValueError):
        NativePlan(net, [(0, 0)], torch.complex64, None, [])
    net_bad = Network([[0, 1], [1, 2]], [0, 2], {0: 2, 1: 3, 2: 2})
    with pytest.raises(ValueError):          # a sliced mode that is an output mode
        NativePlan(net_bad, [(0, 1)], torch.complex64, None, [0])


@pytest.mark.parametrize("n_legs,want_s2", [(24, True), (34, False)])
def test_sweep2_lane_offsets_stay_32bit(n_legs, want_s2):
    """SWEEP2 carries a lane's load/store offset (the low 9 chunk bits of its enumeration) as a
    32-bit byte offset (csrc/tq_sweep2.hip lane_at).  A chain of 4 two-leg gates on the 8
    highest-order legs of a 2^n_legs complex64 tensor puts tile bits of stride 2^(n-8)..2^(n-5)
    among those low bits: at n = 34 they reach 2^32 bytes and the plan must not use SWEEP2
    (it falls back to per-gate APPLY); at n = 24 it does."""
    import torch
    from tneq_qc_amd.einsum import get_symbol
    from tneq_qc_amd.expression import HipContractExpression
    legs = [get_symbol(i) for i in range(n_legs)]
    terms = ["".join(legs)]
    cur = list(legs)
    nxt = n_legs
    for g in range(4):
        a, b = cur[2 * g], cur[2 * g + 1]
        na, nb = get_symbol(nxt), get_symbol(nxt + 1)
        nxt += 2
        terms.append(a + b + na + nb)
        cur[2 * g], cur[2 * g + 1] = na, nb
    eq = ",".join(terms) + "->" + "".join(cur)
    shapes = [(2,) * n_legs] + [(2, 2, 2, 2)] * 4
    path = [(0, 1)] + [(5 + i, 2 + i) for i in range(3)]
    e = HipContractExpression(eq, *shapes, optimize=path)
    d = e.plan(torch.complex64).describe()
    assert ("SWEEP2" in d) == want_s2, d


@pytest.mark.parametrize("cfg", ["C3", "C4g"])
def test_boundary_gemm_takes_presplit_operands(cfg):
    """The boundary GEMM of C3 / C4 is a pre-split candidate: both operands come from per-slice
    sweep2 ops that nothing else reads, so those ops may store the f16 terms the GEMM consumes
    (tq_plan.cpp Compiler::assign_amax); the operand-max words stay in place for the check."""
    e, p = _plan(config_task(cfg))
    gemm = [l for l in p.describe().splitlines() if " GEMM " in l]
    assert len(gemm) == 1 and "amax<-" in gemm[0]
    if cfg == "C4g":
        # C4g's operands come from dense producers, which store the six f16 term planes of the
        # pre-split GEMM instead (tq_gemmp.hip; the planes GEMM replaces the presplit form)
        assert p.query("n_presplit") == 0 and p.query("planes_gemm") == 1 and " planes " in gemm[0]
        assert "planes(A)" in p.describe() and "planes(B)" in p.describe()
    else:
        assert p.query("n_presplit") == 1 and "presplit" in gemm[0] and p.query("planes_gemm") == 0
    # complex128 plans have no f16 path and no candidates
    e2, p2 = _plan(config_task(cfg), "complex128")
    assert p2.query("n_presplit") == 0


def test_slice_lanes_within_the_arena_budget():
    """Slices run in batches of `lanes` (a power of two) within an arena budget (C3: 64
    latency-bound slices, 32 per batch, each lane with its own copy of the per-slice buffers);
    C4's 1.1-GiB per-slice part gets 4 (the lane copies stay within 6 GiB; tq_plan.cpp, Plan::lanes)."""
    e3, p3 = _plan(config_task("C3"))
    assert p3.query("lanes") == 32
    e4, p4 = _plan(config_task("C4g"))
    assert p4.query("lanes") == 4   # 1.1-GiB per-slice part: 4 lanes in the 6-GiB budget
    e2, p2 = _plan(config_task("C2"))
    assert p2.query("lanes") == 1   # one slice


def test_small_hoisted_levels_run_as_one_chain_launch():
    """Consecutive hoisted levels of small sweep2 ops (the whole tensor fits one 64-KiB tile and
    the default layout has at most 2 chunks) run as one chain launch, a workgroup per stream
    (tq_plan.cpp Plan::seq_once): the first levels of C2, C3 and C4 (C3 / C4: the left and right
    halves on streams of their own); consecutive ops of a stream hand their tensor over in LDS.
    C2's later 4-chunk levels stay one launch each (measured faster, tq_plan.cpp
    s2_seq_max_chunks); "sweep_chain" = 0 restores one launch per level."""
    for cfg in ("C2", "C3", "C4g"):
        e, p = _plan(config_task(cfg))
        d = [l for l in p.describe().splitlines() if l.startswith("# chain launch")]
        assert len(d) == 1 and "<" in d[0] and ">" in d[0], d
        assert ("/s1" in d[0]) == (cfg != "C2")
        n_on = p.query("n_launch_once")
        ops = d[0].split("ops")[1].split("(")[0].split()
        levels = int(d[0].split("..")[1].split(",")[0]) - int(d[0].split("entries ")[1].split("..")[0]) + 1
        assert p.query("n_chain_launches") == 1 and levels >= 2 and len(ops) >= (2 if cfg == "C2" else 4)
        p.set("sweep_chain", 0)
        assert p.query("n_chain_launches") == 0 and p.query("n_launch_once") == n_on + levels - 1
        p.set("sweep_chain", 1)


def test_multi_chunk_hoisted_levels_run_as_one_cooperative_launch():
    """C2's hoisted levels of one multi-chunk sweep2 op each (after its one-chunk chain) form
    ONE cooperative launch of 8 workgroups (its most common chunk count) with a counter barrier
    between the ops (tq_plan.cpp Plan::coop_once), run when "sweep_coop" = 1 (measured slower,
    so off by default: one launch per level).  C3 / C4 have no such run (their multi-chunk levels
    hold several ops or are per slice)."""
    e, p = _plan(config_task("C2"))
    assert p.query("n_coop_launches") == 0   # off by default
    p.set("sweep_coop", 1)
    d = [l for l in p.describe().splitlines() if l.startswith("# cooperative chain launch")]
    assert len(d) == 1 and "(8 workgroups" in d[0], d
    ops = [int(x) for x in d[0].split(", ops")[1].split()]
    assert ops == list(range(ops[0], ops[0] + len(ops))) and len(ops) >= 20
    assert p.query("n_coop_launches") == 1 and p.query("n_coop_ops") == len(ops)
    n_on = p.query("n_launch_once")
    p.set("sweep_coop", 0)
    assert p.query("n_coop_launches") == 0 and p.query("n_launch_once") == n_on + len(ops) - 1
    p.set("sweep_coop", 1)
    for cfg in ("C3", "C4g"):
        assert _plan(config_task(cfg))[1].query("n_coop_launches") == 0


@pytest.mark.parametrize("cfg", ["C3", "C4g"])
def test_lane_batched_boundary_gemm_and_lane_sum(cfg):
    """With slice lanes the boundary GEMM (lane-local operands) is one batched launch per batch
    (`lanes`), and since only the output permute reads its result the lanes' results are summed
    before that permute runs once (`lane-sum`; tq_plan.cpp Op::lane_batch / lane_sum)."""
    e, p = _plan(config_task(cfg))
    d = p.describe().splitlines()
    gemm = [l for l in d if " GEMM " in l]
    assert len(gemm) == 1 and " lanes" in gemm[0] and "lane-sum" in gemm[0]
    perm = [l for l in d if "PERMUTE result->out" in l]
    assert len(perm) == 1 and "[slice]" in perm[0]


@pytest.mark.parametrize("cfg,legacy,gain", [("C4", "C4g", 100.0), ("C3d", "C3", 5.0)])
def test_deferred_tails_shrink_the_boundary(cfg, legacy, gain):
    """The deferred C3d / C4 paths absorb the last tensors of each half's sweep after the
    boundary contraction (einsum.partition_path(defer=...)): the boundary GEMM contracts only the
    cut legs those expanding gates do not touch.  Same network, same amplitudes (GPU parity:
    tests/test_fullsize_gpu.py); the complex-MAC count drops by `gain` or more and the boundary
    GEMM becomes slice-invariant (hoisted, run once per execute)."""
    from tneq_qc_amd import einsum as E
    t, tg = config_task(cfg), config_task(legacy)
    assert t.eq == tg.eq and t.path != tg.path
    net = E.parse_equation(t.eq, t.shapes)
    E.validate_path(len(net.terms), t.path)
    f = E.path_info(net, t.path, [net.symbols.index(x) for x in t.sliced]).flops
    fg = E.path_info(net, tg.path, [net.symbols.index(x) for x in tg.sliced]).flops
    assert f * gain <= fg, (f, fg)
    e, p = _plan(t)
    gemm = [l for l in p.describe().splitlines() if " GEMM " in l]
    assert len(gemm) == 1 and gemm[0].startswith("[once]"), gemm


def test_partition_path_defer_counts():
    """partition_path(defer=(l, r)) keeps the first len - l (len - r) tensors of each half's sweep,
    contracts the two half results, then absorbs the deferred tensors; defer=(0, 0) is the plain
    partition path, and every deferred path is a valid pairwise path of the same network."""
    from tneq_qc_amd import einsum as E
    from tneq_qc_amd.circuits import BrickWall, amplitude_task
    t0 = amplitude_task(BrickWall(12, 6, 0), list(range(4, 8)), cut=6)
    t1 = amplitude_task(BrickWall(12, 6, 0), list(range(4, 8)), cut=6, defer=(0, 0))
    assert t0.path == t1.path
    net = E.parse_equation(t0.eq, t0.shapes)
    for d in ((2, 0), (0, 3), (4, 4)):
        t = amplitude_task(BrickWall(12, 6, 0), list(range(4, 8)), cut=6, defer=d)
        E.validate_path(len(net.terms), t.path)
        assert t.path != t0.path
        # the boundary contraction (the step joining the two halves) comes sum(d) steps before the end
        assert len(t.path) == len(t0.path)


def test_deferred_paths_contract_to_the_same_amplitudes():
    """Every deferred split of a small cut network is a valid pairwise path of the same network and
    the oracle's contraction along it gives the plain partition path's amplitudes (sliced sums
    included); einsum.deferred_search's pick costs no more than the plain path in the model."""
    import numpy as np
    from oracle.contract_ref import contract_sliced
    from tneq_qc_amd import einsum as E
    from tneq_qc_amd.circuits import BrickWall, amplitude_task
    circ = BrickWall(12, 6, 4)
    t0 = amplitude_task(circ, list(range(4, 8)), cut=6, n_slice=2)
    ref = contract_sliced(t0.eq, t0.operands, t0.sliced, t0.path)
    net = E.parse_equation(t0.eq, t0.shapes)
    for d in ((2, 2), (4, 0), (0, 4), (6, 6)):
        t = amplitude_task(circ, list(range(4, 8)), cut=6, n_slice=2, defer=d)
        assert t.eq == t0.eq
        E.validate_path(len(net.terms), t.path)
        got = contract_sliced(t.eq, t.operands, t.sliced, t.path)
        assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max(), d
    ta = amplitude_task(circ, list(range(4, 8)), cut=6, n_slice=2, defer="auto")
    sl = lambda t: [net.symbols.index(x) for x in t.sliced]
    assert E.path_info(net, ta.path, sl(ta)).est_seconds <= E.path_info(net, t0.path, sl(t0)).est_seconds * (1 + 1e-9)
    got = contract_sliced(ta.eq, ta.operands, ta.sliced, ta.path)
    assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max()


def test_branches_follow_the_boundary_join():
    """With deferred tails the final step joins a tail gate, not the two halves: the plan's two
    branches (own arena regions, tq_plan.cpp branches pre-pass) must still be the halves, so their
    hoisted sweep levels share launches (C4: most hoisted launches hold one op of each half)."""
    e, p = _plan(config_task("C4"))
    d = p.describe().splitlines()
    ops = [l for l in d if l.startswith("[once]") or l.startswith("[slice]")]
    assert any(" b0 " in l for l in ops) and any(" b1 " in l for l in ops)
    pairs = 0
    for l in d:
        if l.startswith("# once"):
            ids = [int(x) for x in l.split()[2:]]
            br = {ops[i].split()[1] for i in ids}
            pairs += len(ids) == 2 and br == {"b0", "b1"}
    assert pairs >= 10, pairs
    # the last per-slice level is lane-merged and read only by the output permute: its lanes are
    # summed before one permute per batch (Op::lane_sum on a sweep2 level)
    assert any(l.startswith("[slice]") and "SWEEP2" in l and "lane-sum" in l for l in ops)


def _old_planes_ws(M, N, K, lanes):
    """The r05 sizing before d90d7cb: the partials of a FULL lane batch only."""
    L = _lib.lib()
    one = L.tq_planes_gemm_workspace(M, N, K, lanes)   # >= the full batch's own need
    # the full batch's own need = 3 x batch x splits(batch) x M x N x 4 bytes: recover it as the
    # smallest workspace the check accepts for `lanes`
    lo, hi = 0, one
    while lo < hi:
        mid = (lo + hi) // 2
        if L.tq_planes_gemm_check(M, N, K, lanes, M, N, mid) == 0:
            hi = mid
        else:
            lo = mid + 1
    return lo


@pytest.mark.parametrize("cfg", ["C4g"])
def test_planes_gemm_workspace_covers_every_lane_batch(cfg):
    """VERDICT r5 item 6 (the r05c GPU fault): the planes GEMM's split-K partials must fit every
    lane-batch size a slice range can produce (a partial batch may pick MORE splits than a full
    one), and the launcher refuses a workspace that is too small -- checked on the host, through
    the same sizing and argument checks the GPU launch runs (tq_planes_gemm_check), no GPU."""
    L = _lib.lib()
    e, p = _plan(config_task(cfg))
    assert p.query("planes_gemm") == 1
    M, N, K = (p.query(f"planes_gemm_{k}") for k in "MNK")
    lda, ldb = p.query("planes_gemm_lda"), p.query("planes_gemm_ldb")
    lanes = p.query("lanes")
    ws = p.query("planes_ws_bytes")
    assert lanes >= 2 and ws > 0
    assert ws >= L.tq_planes_gemm_workspace(M, N, K, lanes)
    for b in range(1, lanes + 1):
        assert L.tq_planes_gemm_check(M, N, K, b, lda, ldb, ws) == 0, (b, _lib.last_error())
    # the pre-fix sizing (the full batch's own partials) is too small for some partial batch
    old = _old_planes_ws(M, N, K, lanes)
    assert any(L.tq_planes_gemm_check(M, N, K, b, lda, ldb, old) != 0 for b in range(1, lanes))
    # the refusal itself: one byte short of a batch's need
    need = max(L.tq_planes_gemm_workspace(M, N, K, b) for b in range(1, lanes + 1))
    worst = [b for b in range(1, lanes + 1) if L.tq_planes_gemm_check(M, N, K, b, lda, ldb, need - 1) != 0]
    assert worst, "some batch size needs the whole workspace"
    assert "exceed the workspace" in _lib.last_error()
    # and unsupported shapes are refused before any sizing
    assert L.tq_planes_gemm_check(M + 1, N, K, 1, lda, ldb, ws) != 0


def test_group_hint_recompiles_with_wider_chunks():
    """A plan compiled for lockstep groups (tq_plan_set "group_hint", BlockPipeline --group):
    the same ops and schedule, sweep ops with fewer, wider chunks (G ops share each launch);
    refused after the first execute; a clone keeps the hint."""
    import torch
    e, p = _plan(config_task("C4"))
    d1 = p.describe()
    n1 = p.query("n_kernels")
    p.set("group_hint", 4)
    assert p.query("group_hint") == 4 and p.query("n_kernels") == n1
    d4 = p.describe()
    chunks = lambda d: sum(int(x) for x in re.findall(r"chunks=(\d+)", d))
    if chunks(d1):
        assert chunks(d4) < chunks(d1)
    q = p.clone()
    assert q.query("group_hint") == 4 and q.query("n_kernels") == n1
    p.set("group_hint", 1)
    assert p.describe() == d1
