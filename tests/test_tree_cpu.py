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
    if not slices:
        return torch.from_numpy(np.ascontiguousarray(contract(eq, *arrs)))
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
