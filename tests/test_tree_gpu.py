"""Partitioned contraction with log2(W) merge stages on the native plan: W = 2 and 4 ranks
(gloo process groups, all on cuda:0; on the 8-GPU node one rank per GPU over RCCL) contract the
C5 ansatz network (symmetry-breaking 8-qubit brick wall, core-only output, complex128) —
stage 0 per-rank partitions, then K-sharded merges + all_reduce — and every rank's result equals
the oracle's unpartitioned contraction (1e-12)."""
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
        from oracle.contract_ref import contract
        from tneq_qc_amd.circuits import ansatz_qctn
        from tneq_qc_amd.contractor import EinsumStrategy
        from tneq_qc_amd.distributed import TreeContraction
        torch.cuda.set_device(0)
        bw = ansatz_qctn()
        q_ = bw.qctn
        eq, shapes = EinsumStrategy.build_core_only_expression(q_)
        ops_np = [bw.cores[c] for c in q_.cores]
        job = TreeContraction(eq, shapes)
        res = job(*[torch.from_numpy(o).to("cuda:0") for o in ops_np]).cpu().numpy()
        full = contract(eq, *ops_np)
        q.put((rank, float(np.abs(res - full).max() / np.abs(full).max())))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_tree_on_native_plans(dev, world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=200)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    for rank, err in (q.get(timeout=5) for _ in range(world)):
        assert err < 1e-12, (rank, err)
