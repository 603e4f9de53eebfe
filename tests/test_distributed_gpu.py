"""N>1 path with the native plan: two ranks (gloo process group, both on cuda:0) each run the
HIP plan on their round-robin slice range (slices r, r+2, ...) through SlicedContraction and
all-reduce the partial amplitudes; rank 0 compares with the oracle's unsliced contraction, and
each rank's partial with the oracle's sum over that rank's slices (complex128, 1e-12).
(On the 8-GPU node the same object runs one rank per GPU with the reduce over RCCL.)"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.contract_ref import contract, sliced_operands
        from tneq_qc_amd.circuits import BrickWall, amplitude_task
        from tneq_qc_amd.distributed import SlicedContraction
        from tneq_qc_amd.expression import HipContractExpression
        torch.cuda.set_device(0)
        task = amplitude_task(BrickWall(12, 6, 2), list(range(4, 8)), cut=6, n_slice=3)
        expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
        ops = [torch.from_numpy(o).to("cuda:0", torch.complex128) for o in task.operands]
        job = SlicedContraction(expr)
        assert (job.rank, job.world) == (rank, world)
        # this rank's partial (before the reduce) vs the oracle over the same slices
        part = expr(*ops, slice_range=(rank, expr.n_slices, world)).cpu().numpy()
        ref_part = 0
        for s in range(rank, expr.n_slices, world):
            eq_s, ops_s = sliced_operands(task.eq, task.operands, task.sliced, s)
            ref_part = ref_part + contract(eq_s, *ops_s)
        perr = float(np.abs(part - ref_part).max() / np.abs(ref_part).max())
        res = job(*ops).cpu().numpy()
        full = contract(task.eq, *task.operands)
        err = float(np.abs(res - full).max() / np.abs(full).max())
        q.put((rank, perr, err))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_ranks_run_the_native_plan_and_reduce(dev):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=200)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0, 0], codes
    got = sorted(q.get(timeout=5) for _ in range(2))
    for rank, perr, err in got:
        assert perr < 1e-12, (rank, perr)
        assert err < 1e-12, (rank, err)
