"""Gradients and TNTensor scales through the multi-GPU paths on the native plans (ranks are gloo
process groups on cuda:0 here; on the 8-GPU node one rank per GPU over RCCL), plus the
DistributedEngineSiamese drop-in against the single-process EngineSiamese, and RCCL itself.

* sliced autograd: HipContractExpression(slices=...) called with a slice range and
  requires-grad operands == torch autograd over the same slices (c128, 1e-10);
* SlicedContraction / TreeContraction at W = 2: the loss is taken on every rank; a rank's
  gradient == W x the single-process gradient (the reference's AllReduceGrad / SendRecvGrad
  adjoints, allreduce_grad.py:13-60, 149-207);
* DistributedEngineSiamese (distributed_engine.py:368-1984) at W = 2 == EngineSiamese
  .contract_with_compiled_strategy (forward) and W x contract_with_compiled_strategy_for_gradient
  (gradients), TNTensor cores included;
* RCCL: a 1-rank "nccl" group initialised exactly as bench.py does, a direct all_reduce of the
  view_as_real complex64 partial buffer, and SlicedContraction over it."""
import os
import socket

import numpy as np
import pytest

from test_distributed_cpu import _torch_slices
from test_tree_cpu import _torch_executor

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(target, world, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=200)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    return sorted(q.get(timeout=5) for _ in range(world))


def _task():
    from tneq_qc_amd.circuits import BrickWall, amplitude_task
    return amplitude_task(BrickWall(8, 4, 2), list(range(2, 6)), cut=4, n_slice=3)


def test_sliced_range_gradients(dev):
    import torch
    from tneq_qc_amd.expression import HipContractExpression
    task = _task()
    expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
    for rng in [(0, expr.n_slices, 1), (1, expr.n_slices, 3), (5, 6, 1)]:
        ts = [torch.tensor(o, dtype=torch.complex128, device=dev, requires_grad=True) for o in task.operands]
        out = expr(*ts, slice_range=rng)
        w = torch.linspace(-1, 1, out.numel(), dtype=torch.float64, device=dev).reshape(out.shape)
        g = torch.autograd.grad((out * w).real.sum() + (out.abs() ** 2).sum(), ts, allow_unused=True)
        rts = [torch.tensor(o, dtype=torch.complex128, requires_grad=True) for o in task.operands]
        ref = _torch_slices(task.eq, task.sliced, rng, rts)
        wc = w.cpu()
        rg = torch.autograd.grad((ref * wc).real.sum() + (ref.abs() ** 2).sum(), rts, allow_unused=True)
        assert (out.detach().cpu() - ref.detach()).abs().max() <= 1e-12 * ref.detach().abs().max()
        scale = max(float(b.abs().max()) for b in rg if b is not None)
        for a, b in zip(g, rg):
            if b is None:
                assert a is None or float(a.abs().max()) == 0.0
                continue
            assert float((a.cpu() - b).abs().max()) <= 1e-10 * scale


def _sliced_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tneq_qc_amd.core import TNTensor
        from tneq_qc_amd.distributed import SlicedContraction
        from tneq_qc_amd.expression import HipContractExpression
        torch.cuda.set_device(0)
        task = _task()
        expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
        job = SlicedContraction(expr)
        ts = [torch.tensor(o, dtype=torch.complex128, device="cuda:0", requires_grad=True) for o in task.operands]
        res = job(*ts)
        w = torch.linspace(-1, 1, res.numel(), dtype=torch.float64, device="cuda:0").reshape(res.shape)
        g = torch.autograd.grad((res * w).real.sum() + (res.abs() ** 2).sum(), ts)
        rts = [torch.tensor(o, dtype=torch.complex128, requires_grad=True) for o in task.operands]
        ref = torch.einsum(task.eq, *rts)
        rg = torch.autograd.grad((ref * w.cpu()).real.sum() + (ref.abs() ** 2).sum(), rts)
        e_out = float((res.detach().cpu() - ref.detach()).abs().max() / ref.detach().abs().max())
        e_g = max(float((a.cpu() - world * b).abs().max()) for a, b in zip(g, rg)) / max(
            float(b.abs().max()) for b in rg)
        tn = [TNTensor(torch.tensor(o / 2.0 ** (9 * (i % 4) - 13), dtype=torch.complex128, device="cuda:0"),
                       2.0 ** (9 * (i % 4) - 13)) for i, o in enumerate(task.operands)]
        r2 = job(*tn)
        e_tn = float(((r2.tensor * r2.scale).cpu() - ref.detach()).abs().max() / ref.detach().abs().max())
        q.put((rank, e_out, e_g, e_tn))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_sliced_contraction_gradients_two_ranks(dev):
    for rank, e_out, e_g, e_tn in _spawn(_sliced_worker, 2):
        assert e_out < 1e-12 and e_g < 1e-10 and e_tn < 1e-12, (rank, e_out, e_g, e_tn)


def _tree_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tneq_qc_amd.circuits import BrickWall
        from tneq_qc_amd.contractor import EinsumStrategy
        from tneq_qc_amd.distributed import TreeContraction
        torch.cuda.set_device(0)
        bw = BrickWall(5, 4, 3)
        eq, shapes = EinsumStrategy.build_core_only_expression(bw.qctn)
        ops = [bw.cores[c] for c in bw.qctn.cores]
        job = TreeContraction(eq, shapes)          # native plans
        ts = [torch.tensor(o, device="cuda:0", requires_grad=True) for o in ops]
        out = job(*ts)
        w = torch.linspace(-1, 1, out.numel(), dtype=torch.float64, device="cuda:0").reshape(out.shape)
        g = torch.autograd.grad((out * w).real.sum() + (out.abs() ** 2).sum(), ts, allow_unused=True)
        rts = [torch.tensor(o, requires_grad=True) for o in ops]
        ref = torch.einsum(eq, *rts)
        rg = torch.autograd.grad((ref * w.cpu()).real.sum() + (ref.abs() ** 2).sum(), rts)
        e_out = float((out.detach().cpu() - ref.detach()).abs().max() / ref.detach().abs().max())
        e_g = max(float((g[t].cpu() - world * rg[t]).abs().max() / rg[t].abs().max()) for t in job.parts[rank])
        q.put((rank, e_out, e_g))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_tree_gradients_native(dev, world):
    for rank, e_out, e_g in _spawn(_tree_worker, world):
        assert e_out < 1e-12 and e_g < 1e-10, (rank, e_out, e_g)


def _engine_setup(dev):
    import torch
    from oracle.qctn_ref import QCTNRef, random_cores
    from tneq_qc_amd.circuits import build_brick_wall_IM, incidence_to_graph
    from tneq_qc_amd.core import QCTN
    g = incidence_to_graph(build_brick_wall_IM(4, 2))
    cores = random_cores(QCTNRef(g), 11)
    q = QCTN(g)
    q.cores_weights = {c: torch.tensor(cores[c], device=dev) for c in q.cores}
    rng = np.random.default_rng(3)
    states = [torch.tensor([1.0, 0.0], dtype=torch.complex128, device=dev) for _ in range(q.nqubits)]
    mx = []
    for _ in range(q.nqubits):
        m = rng.standard_normal((3, 2, 2)) + 1j * rng.standard_normal((3, 2, 2))
        mx.append(torch.tensor(m + np.conj(np.swapaxes(m, 1, 2)), device=dev))
    return q, cores, states, mx


def _engine_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tneq_qc_amd.backends import BackendFactory
        from tneq_qc_amd.core import TNTensor
        from tneq_qc_amd.core.engine_siamese import EngineSiamese
        from tneq_qc_amd.distributed import DistributedEngineSiamese
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        backend = BackendFactory.create_backend("hip", device="cuda:0", dtype="complex128")
        qc, cores, states, mx = _engine_setup(dev)
        single = EngineSiamese(backend, "balanced")
        ref = single.contract_with_compiled_strategy(qc, states, mx).cpu()
        qc2, _, _, _ = _engine_setup(dev)
        for c in qc2.cores:
            qc2.cores_weights[c].requires_grad_(True)
        ref_loss, ref_g = single.contract_with_compiled_strategy_for_gradient(qc2, states, mx)
        ref_g = dict(zip(qc2.cores, ref_g))
        eng = DistributedEngineSiamese(backend)
        eng.init_distributed(qc)
        res = eng.contract_distributed(states, mx).cpu()
        e_fwd = float((res - ref).abs().max() / ref.abs().max())
        loss, grads = eng.contract_distributed_with_gradient(states, mx)
        e_loss = abs(float(loss) - float(ref_loss)) / abs(float(ref_loss))
        e_g = max(float((gr - world * ref_g[c]).abs().max() / ref_g[c].abs().max())
                  for c, gr in zip(eng._local_qctn.cores, grads))
        scales = {c: 2.0 ** (5 * (i % 4) - 7) for i, c in enumerate(qc.cores)}
        qc3, _, _, _ = _engine_setup(dev)
        qc3.cores_weights = {c: TNTensor(qc3.cores_weights[c] / scales[c], scales[c]) for c in qc3.cores}
        single_tn = single.contract_with_compiled_strategy(qc3, states, mx, ret_type="TNTensor")
        eng.init_distributed(qc3)
        with torch.no_grad():
            r3 = eng.contract_distributed(states, mx)
        e_tn = float(((r3.tensor * r3.scale).cpu() - (single_tn.tensor * single_tn.scale).cpu()).abs().max()
                     / (single_tn.tensor * single_tn.scale).abs().max().cpu())
        q.put((rank, e_fwd, e_loss, e_g, e_tn))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_distributed_engine_native_two_ranks(dev):
    for rank, e_fwd, e_loss, e_g, e_tn in _spawn(_engine_worker, 2):
        assert e_fwd < 1e-12 and e_loss < 1e-12 and e_g < 1e-10 and e_tn < 1e-12, (rank, e_fwd, e_loss, e_g, e_tn)


def _rccl_worker(rank, world, port, q):
    """A 1-rank RCCL group initialised exactly as bench.py (init_process_group("nccl",
    device_id=dev)); a direct all_reduce of the view_as_real complex64 buffer (allreduce_partials
    short-circuits at world 1, so the collective is called here directly) and the
    SlicedContraction bench path over the group."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    try:
        from tneq_qc_amd.distributed import SlicedContraction
        from tneq_qc_amd.expression import HipContractExpression
        assert dist.get_backend() == "nccl"
        x = (torch.randn(1 << 16, dtype=torch.complex64, device=dev))
        y = x.clone()
        dist.all_reduce(torch.view_as_real(y), op=dist.ReduceOp.SUM)
        torch.cuda.synchronize()
        e_ar = float((y - x).abs().max())
        m = torch.tensor([3.5], dtype=torch.float64, device=dev)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        task = _task()
        expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
        ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in task.operands]
        out = torch.empty(expr.out_shape, dtype=torch.complex64, device=dev)
        res = SlicedContraction(expr)(*ops, out=out).cpu().numpy()
        from oracle.contract_ref import contract
        full = contract(task.eq, *task.operands)
        e_sc = float(np.abs(res - full).max() / np.abs(full).max())
        dist.barrier()
        q.put((rank, e_ar, float(m.item()), e_sc))
    finally:
        dist.destroy_process_group()


def test_rccl_one_rank_all_reduce(dev):
    (rank, e_ar, mx, e_sc), = _spawn(_rccl_worker, 1)
    assert e_ar == 0.0 and mx == 3.5 and e_sc < 2e-5, (e_ar, mx, e_sc)


def _comm_engine_worker(rank, world, port, q):
    """The reference trainer's construction (distributed_trainer.py:228-233, 271-283) on one GPU:
    comm = get_comm_backend('torch'), then DistributedEngineSiamese(backend=..., strategy_mode=...,
    mx_K=..., comm=comm, partition_config=...) on the HIP backend, against the single-process
    EngineSiamese -- first as the trainer runs at world 1 (CommTorch, like comm_torch.py:140-175,
    initialises no group there), then joining a 1-rank "nccl" (RCCL) group initialised as the
    launcher / bench.py does, with CommTorch's allreduce of a complex64 device tensor over it."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    from tneq_qc_amd.backends import BackendFactory
    from tneq_qc_amd.core.engine_siamese import EngineSiamese
    from tneq_qc_amd.distributed import DistributedEngineSiamese, PartitionConfig, ReduceOp, get_comm_backend
    backend = BackendFactory.create_backend("hip", device="cuda:0", dtype="complex128")
    qc, cores, states, mx = _engine_setup(dev)
    ref = EngineSiamese(backend, "balanced").contract_with_compiled_strategy(qc, states, mx).cpu()

    def run(comm):
        eng = DistributedEngineSiamese(backend=backend, strategy_mode="balanced", mx_K=100, comm=comm,
                                       partition_config=PartitionConfig(num_partitions=comm.world_size))
        same = eng.comm is comm and (eng.rank, eng.world_size) == (0, 1)
        eng.init_distributed(qc)
        res = eng.contract_distributed(states, mx).cpu()
        return same, float((res - ref).abs().max() / ref.abs().max())

    comm0 = get_comm_backend("torch")
    local = (comm0.is_initialized(),) + run(comm0)
    dist.init_process_group("nccl", device_id=dev)
    comm = get_comm_backend("torch")
    try:
        z = torch.randn(1 << 12, dtype=torch.complex64, device=dev)
        e_ar = float((comm.allreduce(z, ReduceOp.SUM) - z).abs().max())
        rccl = (comm.is_initialized(), dist.get_backend()) + run(comm)
        comm.barrier()
        q.put((rank, local, rccl, e_ar))
    finally:
        comm.destroy()


def test_reference_comm_engine_rccl_one_rank(dev):
    (rank, local, rccl, e_ar), = _spawn(_comm_engine_worker, 1)
    assert local[0] is False and local[1] and local[2] < 1e-12, local
    assert rccl[:3] == (True, "nccl", True) and rccl[3] < 1e-12 and e_ar == 0.0, (rccl, e_ar)
