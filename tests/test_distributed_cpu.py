"""N>1 path on CPU: world_size-2 gloo run of the slice sharding + SUM all-reduce of
tneq_qc_amd.distributed (the per-slice contraction is the oracle here, injected as executor;
on the GPU the same object runs the native plan and the reduce goes over RCCL)."""
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


def _slice_operands(task, slice_id):
    """Operands with the sliced symbols fixed to the digits of slice_id (row-major)."""
    terms = task.eq.split("->")[0].split(",")
    vals, rem = {}, slice_id
    for s in reversed(task.sliced):
        vals[s] = rem % 2
        rem //= 2
    ops = []
    for term, op in zip(terms, task.operands):
        idx = tuple(vals[ch] if ch in vals else slice(None) for ch in term)
        ops.append(np.ascontiguousarray(op[idx]))
    nterms = ["".join(ch for ch in term if ch not in vals) for term in terms]
    return ",".join(nterms) + "->" + task.eq.split("->")[1], ops


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.contract_ref import contract
    from tneq_qc_amd.circuits import BrickWall, amplitude_task
    from tneq_qc_amd.distributed import SlicedContraction, shard_slices

    task = amplitude_task(BrickWall(12, 6, 2), list(range(4, 8)), cut=6, n_slice=3)

    class _Expr:  # what SlicedContraction needs from an expression
        n_slices = 2 ** len(task.sliced)

    def executor(rng, out):
        b, e, st = rng
        acc = np.zeros((2,) * len(task.open_qubits), complex)
        for s in range(b, e, st):
            eq, ops = _slice_operands(task, s)
            acc += contract(eq, *ops)
        return torch.from_numpy(acc)

    job = SlicedContraction(_Expr(), executor=executor)
    assert (job.rank, job.world) == (rank, world)
    assert shard_slices(8, rank, world) == (rank, 8, world)
    res = job().numpy()
    # async reduce (bench.py's pipelined steps): (result, work), the sum lands after work.wait()
    res2, work = job(async_reduce=True)
    assert work is not None
    work.wait()
    with pytest.raises(ValueError):   # autograd / TNTensor operands keep the synchronous reduce
        job(torch.ones(1, requires_grad=True), async_reduce=True)
    if rank == 0:
        full = contract(task.eq, *task.operands)
        q.put(max(float(np.abs(res - full).max() / np.abs(full).max()),
                  float(np.abs(res2.numpy() - full).max() / np.abs(full).max())))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_slice_sum_equals_full_contraction():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) < 1e-12


def test_allreduce_with_grad_single_process_is_identity():
    from tneq_qc_amd.distributed import allreduce_with_grad
    x = torch.randn(4, dtype=torch.complex128, requires_grad=True)
    y = allreduce_with_grad(x)
    (y.abs() ** 2).sum().backward()
    assert torch.allclose(x.grad, 2 * x.detach())


def _torch_slices(eq, sliced, rng, tensors):
    """Differentiable per-slice executor (torch.einsum on `select` views, slice ids row-major
    over `sliced` as tq_plan_execute enumerates them)."""
    lhs, rhs = eq.split("->")
    terms = lhs.split(",")
    sub = ",".join("".join(c for c in t if c not in sliced) for t in terms) + "->" + rhs
    b, e, st = rng
    acc = None
    for sid in range(b, e, st):
        vals, rem = {}, sid
        for c in reversed(sliced):
            vals[c] = rem % 2
            rem //= 2
        views = []
        for t, o in zip(terms, tensors):
            v = o
            for ax in reversed(range(len(t))):
                if t[ax] in vals:
                    v = v.select(ax, vals[t[ax]])
            views.append(v)
        r = torch.einsum(sub, *views)
        acc = r if acc is None else acc + r
    return acc


def _grad_worker(rank, world, port, q):
    """Gradients through the slice sharding + AllReduceSum (allreduce_grad.py:13-60): every
    rank takes the same loss of the replicated amplitudes; a rank's gradient is that of the
    sum of the ranks' losses (world x the single-process gradient), exactly as the reference's
    AllReduceGrad adjoint gives.  TNTensor operands: the per-rank partials are normalised, their
    log-scales aligned by an all_reduce(MAX) and the result is a TNTensor of the same value."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tneq_qc_amd.circuits import BrickWall, amplitude_task
    from tneq_qc_amd.core.tn_tensor import TNTensor
    from tneq_qc_amd.distributed import SlicedContraction
    task = amplitude_task(BrickWall(8, 4, 2), list(range(2, 6)), cut=4, n_slice=3)

    class _Expr:
        n_slices = 2 ** len(task.sliced)

    def executor(rng, out, *tensors):
        return _torch_slices(task.eq, task.sliced, rng, tensors)

    job = SlicedContraction(_Expr(), executor=executor)
    ts = [torch.tensor(o, dtype=torch.complex128, requires_grad=True) for o in task.operands]
    res = job(*ts)
    w = torch.linspace(-1, 1, res.numel(), dtype=torch.float64).reshape(res.shape)
    loss = (res * w).real.sum() + (res.abs() ** 2).sum()
    g = torch.autograd.grad(loss, ts)
    ref_ts = [torch.tensor(o, dtype=torch.complex128, requires_grad=True) for o in task.operands]
    ref = torch.einsum(task.eq, *ref_ts)
    ref_g = torch.autograd.grad((ref * w).real.sum() + (ref.abs() ** 2).sum(), ref_ts)
    err_out = float((res.detach() - ref.detach()).abs().max() / ref.detach().abs().max())
    err_g = max(float((a - world * b).abs().max()) for a, b in zip(g, ref_g)) / max(
        float(b.abs().max()) for b in ref_g)
    # TNTensor operands (scales 2^-20 .. 2^20, one negative)
    tn = []
    for i, o in enumerate(task.operands):
        sc = 2.0 ** (10 * (i % 5) - 20) * (-1 if i == 3 else 1)
        tn.append(TNTensor(torch.tensor(o / sc, dtype=torch.complex128), scale=sc))
    with torch.no_grad():
        r2 = job(*tn)
    val = r2.tensor * r2.scale
    err_tn = float((val - ref.detach()).abs().max() / ref.detach().abs().max())
    q.put((rank, err_out, err_g, err_tn, isinstance(r2, TNTensor)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_slice_gradients_and_scales():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank, err_out, err_g, err_tn, is_tn in sorted(q.get(timeout=5) for _ in range(2)):
        assert err_out < 1e-12 and err_g < 1e-10 and err_tn < 1e-12 and is_tn, (rank, err_out, err_g, err_tn)


def _few_slices_worker(rank, world, port, q):
    """More ranks than slices (3 ranks, 2 slices): the rank without a slice still joins the
    backward's collectives with a zero partial; gradients are world x the single-process ones."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tneq_qc_amd.circuits import BrickWall, amplitude_task
    from tneq_qc_amd.distributed import SlicedContraction
    task = amplitude_task(BrickWall(8, 4, 2), list(range(2, 6)), cut=4, n_slice=1)

    class _Expr:
        n_slices = 2 ** len(task.sliced)
        out_shape = (2,) * len(task.open_qubits)

    def executor(rng, out, *tensors):
        return _torch_slices(task.eq, task.sliced, rng, tensors)

    job = SlicedContraction(_Expr(), executor=executor)
    ts = [torch.tensor(o, dtype=torch.complex128, requires_grad=True) for o in task.operands]
    res = job(*ts)
    g = torch.autograd.grad((res.abs() ** 2).sum(), ts)
    rts = [torch.tensor(o, dtype=torch.complex128, requires_grad=True) for o in task.operands]
    ref = torch.einsum(task.eq, *rts)
    rg = torch.autograd.grad((ref.abs() ** 2).sum(), rts)
    err = max(float((a - world * b).abs().max()) for a, b in zip(g, rg)) / max(float(b.abs().max()) for b in rg)
    q.put((rank, float((res.detach() - ref.detach()).abs().max()), err))
    dist.barrier()
    dist.destroy_process_group()


def test_more_ranks_than_slices_gradients():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_few_slices_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank, e_out, e_g in sorted(q.get(timeout=5) for _ in range(3)):
        assert e_out < 1e-12 and e_g < 1e-10, (rank, e_out, e_g)


def test_bitstring_blocks_partition_the_state():
    """bench.py's bitstring sharding (circuits.with_batch): block b fixes the closed qubits to the
    base bits flipped by b's binary digits -- the same equation, shapes, path and slicing (one
    plan for every block), only the projector operands differ; a fresh amplitude_task with those
    bits builds the same operands; and the 2^closed blocks are disjoint and cover the state:
    sum over every block of sum |amp|^2 = 1 (a unitary circuit on |0...0>)."""
    from oracle.contract_ref import contract_sliced
    from tneq_qc_amd.circuits import BrickWall, amplitude_task, with_batch
    circ = BrickWall(9, 4, 3)
    opn = list(range(3, 7))
    t = amplitude_task(circ, opn, cut=4, n_slice=2, defer=(2, 2))
    n_closed = len(t.fixed_bits)
    total = 0.0
    seen = set()
    for b in range(2 ** n_closed):
        tb = with_batch(t, b)
        assert tb.eq == t.eq and tb.shapes == t.shapes and tb.path == t.path and tb.sliced == t.sliced
        bits = tuple(sorted(tb.fixed_bits.items()))
        assert bits not in seen
        seen.add(bits)
        if b in (0, 1, 2 ** n_closed - 1):
            fresh = amplitude_task(circ, opn, fixed_bits=tb.fixed_bits, cut=4, n_slice=2, defer=(2, 2))
            assert fresh.eq == tb.eq
            assert all(np.array_equal(x, y) for x, y in zip(fresh.operands, tb.operands))
        amp = contract_sliced(tb.eq, tb.operands, tb.sliced, tb.path)
        total += float((np.abs(amp) ** 2).sum())
    assert abs(total - 1.0) < 1e-10, total
    with pytest.raises(ValueError):
        with_batch(t, 2 ** n_closed)


def _bitstring_worker(rank, world, port, q):
    """bench.py --shard bitstrings on CPU: rank r contracts block r on its own (no collective on
    the data path); the test gathers the blocks only to check them."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.contract_ref import contract_sliced
    from tneq_qc_amd.circuits import BrickWall, amplitude_task, with_batch
    base = amplitude_task(BrickWall(12, 6, 2), list(range(4, 8)), cut=6, n_slice=3)
    mine = with_batch(base, rank)
    amp = torch.from_numpy(contract_sliced(mine.eq, mine.operands, mine.sliced, mine.path))
    got = [torch.zeros_like(amp) for _ in range(world)]
    dist.all_gather(got, amp)
    if rank == 0:
        err = 0.0
        for r in range(world):
            tr = with_batch(base, r)
            ref = contract_sliced(tr.eq, tr.operands, tr.sliced, tr.path)
            err = max(err, float(np.abs(got[r].numpy() - ref).max() / np.abs(ref).max()))
        q.put(err)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_bitstring_blocks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bitstring_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) == 0.0
