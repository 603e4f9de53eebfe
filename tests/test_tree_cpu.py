"""Partitioned contraction with log2(W) merge stages (distributed/tree.py) on CPU: gloo
process groups of 2, 3 and 4 ranks, the per-(sub)network contraction injected as the oracle's
numpy executor (the GPU suite runs the same object on the native plan).  The result on every
rank equals the unpartitioned contraction; the partition rule follows
distributed_engine.py:415-457."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_executor(eq, shapes, operands, slices, slice_range):
    from oracle.contract_ref import contract, sliced_operands
    arrs = [o.numpy() for o in operands]
    if not slices:   # one slice: only range member 0 contracts it (as the native path)
        r = contract(eq, *arrs)
        if slice_range is not None and slice_range[0] >= 1:
            r = np.zeros_like(r)
        return torch.from_numpy(np.ascontiguousarray(r))
    lhs = eq.split("->")[0].split(",")
    ext = {}
    for t, a in zip(lhs, arrs):
        for c, e in zip(t, a.shape):
            ext[c] = e
    n = int(np.prod([ext[c] for c in slices]))
    b, e, st = slice_range
    e = n if e is None else e
    acc = None
    for sid in range(b, e, st):
        eq_s, ops = sliced_operands(eq, arrs, slices, sid)
        r = contract(eq_s, *ops)
        acc = r if acc is None else acc + r
    if acc is None:
        out_shape = tuple(ext[c] for c in eq.split("->")[1])
        acc = np.zeros(out_shape, dtype=np.result_type(*arrs))
    return torch.from_numpy(np.ascontiguousarray(acc))


def _network():
    from tneq_qc_amd.circuits import BrickWall
    from tneq_qc_amd.contractor import EinsumStrategy
    bw = BrickWall(5, 4, 3)
    eq, shapes = EinsumStrategy.build_core_only_expression(bw.qctn)
    return eq, shapes, [bw.cores[c] for c in bw.qctn.cores]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.contract_ref import contract
        from tneq_qc_amd.distributed import TreeContraction
        eq, shapes, ops = _network()
        job = TreeContraction(eq, shapes, executor=_oracle_executor)
        res = job(*[torch.from_numpy(o) for o in ops]).numpy()
        full = contract(eq, *ops)
        q.put((rank, float(np.abs(res - full).max() / np.abs(full).max()), job.n_stages))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_tree_contraction_equals_full(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = [q.get(timeout=5) for _ in range(world)]
    for rank, err, n_stages in got:
        assert err < 1e-12, (rank, err)
        assert n_stages == {2: 1, 3: 2, 4: 2}[world]


def _sub_worker(rank, world, port, q):
    """World of 4: ranks 0-2 run a TreeContraction on their own subgroup (stage exchanges are
    point-to-point inside it: no per-stage process groups), rank 3 never constructs one; two
    instances on the same layout in a row."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.contract_ref import contract
        from tneq_qc_amd.distributed import TreeContraction
        sub = dist.new_group([0, 1, 2])   # every world rank enters the subgroup's own creation
        if rank < 3:
            eq, shapes, ops = _network()
            full = contract(eq, *ops)
            errs = []
            for _ in range(2):
                job = TreeContraction(eq, shapes, group=sub, executor=_oracle_executor)
                res = job(*[torch.from_numpy(o) for o in ops]).numpy()
                errs.append(float(np.abs(res - full).max() / np.abs(full).max()))
            q.put((rank, max(errs)))
        else:
            q.put((rank, 0.0))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_tree_contraction_on_a_subgroup():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sub_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = sorted(q.get(timeout=5) for _ in range(4))
    for rank, err in got:
        assert err < 1e-12, (rank, err)


def test_partition_rule_matches_reference():
    from tneq_qc_amd.distributed import partition_terms
    assert partition_terms(35, 4) == [list(range(0, 9)), list(range(9, 18)), list(range(18, 27)),
                                      list(range(27, 35))]
    assert partition_terms(3, 4) == [[0], [1], [2], []]
    assert partition_terms(6, 2, [[0, 2, 4], [1, 3, 5]]) == [[0, 2, 4], [1, 3, 5]]


def _torch_executor(eq, shapes, operands, slices, slice_range):
    """Differentiable stand-in for the native plan on CPU: torch.einsum per slice on `select`
    views (the same slice enumeration as tq_plan_execute: row-major over `slices`)."""
    lhs, rhs = eq.split("->")
    terms = lhs.split(",")
    if not slices:   # one slice: only range member 0 contracts it (as the native path)
        r = torch.einsum(eq, *operands)
        return r if slice_range is None or slice_range[0] < 1 else torch.zeros_like(r)
    ext = {}
    for t, o in zip(terms, operands):
        for c, e in zip(t, o.shape):
            ext[c] = e
    n = int(np.prod([ext[c] for c in slices]))
    b, e, st = slice_range
    e = n if e is None else e
    sub = ",".join("".join(c for c in t if c not in slices) for t in terms) + "->" + rhs
    acc = None
    for sid in range(b, e, st):
        vals, rem = {}, sid
        for c in reversed(slices):
            vals[c] = rem % ext[c]
            rem //= ext[c]
        views = []
        for t, o in zip(terms, operands):
            v = o
            for ax in reversed(range(len(t))):
                if t[ax] in vals:
                    v = v.select(ax, vals[t[ax]])
            views.append(v)
        r = torch.einsum(sub, *views)
        acc = r if acc is None else acc + r
    if acc is None:
        acc = torch.zeros(tuple(ext[c] for c in rhs), dtype=operands[0].dtype)
    return acc


def _loss(out, w):
    return (out * w).real.sum() + (out.abs() ** 2).sum()


def _grad_worker(rank, world, port, q):
    """Gradients through the tree (the reference's contract_distributed_with_gradient pipeline):
    every rank computes the same loss on the replicated result; the gradient a rank gets for its
    own operands is that of the sum of the ranks' losses = world x the single-process gradient
    (distributed_engine.py:1866-1984 with AllReduceGrad / SendRecvGrad adjoints)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tneq_qc_amd.distributed import TreeContraction
        eq, shapes, ops = _network()
        rng = np.random.default_rng(7)
        job = TreeContraction(eq, shapes, executor=_torch_executor)
        oshape = [job.net.extents[m] for m in job.net.out]
        w = torch.tensor(rng.standard_normal(oshape) + 1j * rng.standard_normal(oshape))
        ts = [torch.tensor(o, requires_grad=True) for o in ops]
        out = job(*ts)
        g = torch.autograd.grad(_loss(out, w), ts, allow_unused=True)
        ref_ts = [torch.tensor(o, requires_grad=True) for o in ops]
        ref_out = torch.einsum(eq, *ref_ts)
        ref_g = torch.autograd.grad(_loss(ref_out, w), ref_ts)
        err_out = float((out.detach() - ref_out.detach()).abs().max())
        errs = []
        for t in job.parts[rank]:
            errs.append(float((g[t] - world * ref_g[t]).abs().max() / ref_g[t].abs().max()))
        # operands of the other partitions are not read on this rank
        unused = all(g[t] is None for p, terms in enumerate(job.parts) if p != rank for t in terms)
        q.put((rank, err_out, max(errs) if errs else 0.0, unused))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_tree_contraction_gradients(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank, err_out, err_g, unused in sorted(q.get(timeout=5) for _ in range(world)):
        assert err_out < 1e-12, (rank, err_out)
        assert err_g < 1e-10, (rank, err_g)
        assert unused, rank


def _scale_worker(rank, world, port, q):
    """TNTensor operands: the scales travel as log-scales through the stages (the reference's
    log-scale exchange + max alignment, distributed_engine.py:1437-1472); the result is a
    TNTensor whose value equals the plain contraction."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.contract_ref import contract
        from tneq_qc_amd.core.tn_tensor import TNTensor
        from tneq_qc_amd.distributed import TreeContraction
        eq, shapes, ops = _network()
        full = contract(eq, *ops)
        tn = []
        for i, o in enumerate(ops):
            s = 2.0 ** (7 * (i % 5) - 14) * (-1 if i % 7 == 3 else 1)
            tn.append(TNTensor(torch.from_numpy(o / s), scale=s))
        job = TreeContraction(eq, shapes, executor=_oracle_executor)
        res = job(*tn)
        assert isinstance(res, TNTensor)
        val = res.tensor.numpy() * np.exp(res.log_scale) * np.sign(res.scale)
        q.put((rank, float(np.abs(val - full).max() / np.abs(full).max())))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_tree_contraction_tntensor_scales(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scale_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank, err in sorted(q.get(timeout=5) for _ in range(world)):
        assert err < 1e-12, (rank, err)


def _empty_part_worker(rank, world, port, q):
    """More ranks than operands (4 ranks, 3 operands): the empty partition is the scalar 1, its
    rank still takes part in every stage and in the backward."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tneq_qc_amd.distributed import TreeContraction
        rng = np.random.default_rng(1)
        eq = "ab,bc,cd->ad"
        shapes = [(3, 4), (4, 5), (5, 2)]
        arrs = [rng.standard_normal(s) + 1j * rng.standard_normal(s) for s in shapes]
        job = TreeContraction(eq, shapes, executor=_torch_executor)
        ts = [torch.tensor(a, requires_grad=True) for a in arrs]
        out = job(*ts)
        extra = [job.leaf] if job.leaf is not None else []
        g = torch.autograd.grad((out.abs() ** 2).sum(), ts + extra, allow_unused=True)
        assert (job.leaf is not None) == (not job.parts[rank])
        rts = [torch.tensor(a, requires_grad=True) for a in arrs]
        ref = torch.einsum(eq, *rts)
        rg = torch.autograd.grad((ref.abs() ** 2).sum(), rts)
        errs = [float((g[t] - world * rg[t]).abs().max() / rg[t].abs().max()) for t in job.parts[rank]]
        q.put((rank, float((out.detach() - ref.detach()).abs().max()), max(errs) if errs else 0.0))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_tree_gradients_with_an_empty_partition():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_empty_part_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank, e_out, e_g in sorted(q.get(timeout=5) for _ in range(4)):
        assert e_out < 1e-12 and e_g < 1e-10, (rank, e_out, e_g)


def _mixed_worker(rank, world, port, q):
    """a rank passes only its own partition (None elsewhere) and only rank 0's
    partition holds TNTensors.  The ranks must agree that log-scales travel (one all-reduce
    MAX on first use): otherwise rank 0 posts scale messages nobody matches (deadlock) or a
    scale is read as payload.  Every rank gets the TNTensor result; a later TNTensor call on a
    contraction agreed unscaled raises on the rank that has one."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.contract_ref import contract
        from tneq_qc_amd.core.tn_tensor import TNTensor
        from tneq_qc_amd.distributed import TreeContraction
        eq, shapes, ops = _network()
        full = contract(eq, *ops)
        job = TreeContraction(eq, shapes, executor=_oracle_executor)
        mine = set(job.parts[rank])
        args = []
        for i, o in enumerate(ops):
            if i not in mine:
                args.append(None)
            elif 0 in mine:
                s = 2.0 ** (5 * (i % 3) - 5)
                args.append(TNTensor(torch.from_numpy(o / s), scale=s))
            else:
                args.append(torch.from_numpy(o))
        res = job(*args)
        assert job.scaled is True
        assert isinstance(res, TNTensor)
        val = res.tensor.numpy() * np.exp(res.log_scale) * np.sign(res.scale)
        err = float(np.abs(val - full).max() / np.abs(full).max())
        # a contraction agreed unscaled refuses TNTensor operands (no unmatched messages)
        plain = TreeContraction(eq, shapes, executor=_oracle_executor)
        r2 = plain(*[torch.from_numpy(o) if i in mine else None for i, o in enumerate(ops)])
        assert plain.scaled is False and not isinstance(r2, TNTensor)
        raised = False
        if 0 in mine:   # it raises before any message (the other ranks do not call)
            try:
                plain(*args)
            except ValueError:
                raised = True
        q.put((rank, err, raised == (0 in mine)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_tree_scales_agreed_with_mixed_partitions(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mixed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank, err, ok in sorted(q.get(timeout=5) for _ in range(world)):
        assert err < 1e-12, (rank, err)
        assert ok, rank
