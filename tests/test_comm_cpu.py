"""The reference's communicator surface (distributed/comm.py) on CPU gloo groups:
  * DistributedEngineSiamese constructed exactly as the reference's trainer does
    (`distributed_trainer.py:228-283`: `comm = get_comm_backend('torch', ...)`, then
    `DistributedEngineSiamese(backend=..., strategy_mode=..., mx_K=..., comm=comm,
    partition_config=...)`) contracts the greedy sandwich equal to the oracle on every rank;
  * CommTorch's collectives (allreduce SUM / AVG / MAX in and out of place, complex tensors,
    allgather, broadcast, broadcast_object, send / recv, isend / irecv, reduce_scatter,
    allreduce_list_async) against their single-process meaning (`comm_torch.py:246-560`);
  * MockCommTorch and the factory's kinds ('mock', 'auto' without a group, 'mpi' refused)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from test_dist_engine_cpu import _setup
from test_tree_cpu import _torch_executor


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from tneq_qc_amd.distributed import DistributedEngineSiamese, PartitionConfig, ReduceOp, get_comm_backend
    comm = get_comm_backend("torch", torch_backend="gloo")
    try:
        out = {"rank": comm.rank, "world": comm.world_size, "init": comm.is_initialized()}
        # collectives
        x = torch.arange(4, dtype=torch.float64) + rank
        out["sum"] = comm.allreduce(x, ReduceOp.SUM).tolist()
        out["avg"] = comm.allreduce(x, ReduceOp.AVG).tolist()
        out["max"] = comm.allreduce(x, ReduceOp.MAX).tolist()
        out["x_unchanged"] = x.tolist()
        z = torch.tensor([1 + 2j, rank * 1j], dtype=torch.complex128)
        comm.allreduce_inplace(z, ReduceOp.SUM)
        out["zsum"] = [complex(v) for v in z]
        out["gather"] = [t.tolist() for t in comm.allgather(torch.tensor([float(rank)]))]
        out["bcast"] = comm.broadcast(torch.tensor([float(rank + 7)]), src=1).tolist()
        out["bobj"] = comm.broadcast_object({"r": rank}, src=0)
        out["rs"] = comm.reduce_scatter(torch.arange(2 * world, dtype=torch.float64), ReduceOp.SUM).tolist()
        h = comm.allreduce_list_async([torch.ones(3) * (rank + 1)], ReduceOp.AVG)
        out["async"] = h.wait()[0].tolist()
        peer = 1 - rank
        buf = torch.zeros(2)
        if rank == 0:
            comm.send(torch.tensor([3.0, 4.0]), peer, tag=5)
            comm.recv(peer, tag=6, tensor=buf)
        else:
            comm.recv(peer, tag=5, tensor=buf)
            comm.send(buf * 10, peer, tag=6)
        out["p2p"] = buf.tolist()
        buf2 = torch.zeros(1)
        w1 = comm.isend(torch.tensor([float(rank)]), peer)
        _, w2 = comm.irecv(peer, tensor=buf2)
        w1.wait()
        w2.wait()
        out["ip2p"] = buf2.tolist()
        comm.barrier()
        # the reference trainer's construction
        from oracle.greedy_ref import greedy_contract
        g, qr, qc, cores, states, mx = _setup()
        eng = DistributedEngineSiamese(backend="hip", strategy_mode="balanced", mx_K=100, comm=comm,
                                       partition_config=PartitionConfig(num_partitions=comm.world_size),
                                       executor=_torch_executor)
        out["eng_rank"] = (eng.rank, eng.world_size, eng.comm is comm)
        qc.cores_weights = {c: torch.tensor(cores[c]) for c in qc.cores}
        eng.init_distributed(qc)
        res = eng.contract_distributed([torch.tensor(s) for s in states], [torch.tensor(m) for m in mx])
        ref = np.abs(greedy_contract(qr, cores, states, mx)) ** 2
        out["err"] = float(np.abs(res.numpy() - ref).max() / np.abs(ref).max())
        out["health"] = eng.check_comm_health()
        q.put(out)
        comm.barrier()
    finally:
        comm.destroy()


def test_engine_with_reference_comm_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = sorted((q.get(timeout=5) for _ in range(world)), key=lambda d: d["rank"])
    for r, o in enumerate(got):
        assert o["rank"] == r and o["world"] == world and o["init"]
        assert o["sum"] == [1.0, 3.0, 5.0, 7.0]
        assert o["avg"] == [0.5, 1.5, 2.5, 3.5]
        assert o["max"] == [1.0, 2.0, 3.0, 4.0]
        assert o["x_unchanged"] == [float(v + r) for v in range(4)]
        assert o["zsum"] == [2 + 4j, 1j]
        assert o["gather"] == [[0.0], [1.0]]
        assert o["bcast"] == [8.0]
        assert o["bobj"] == {"r": 0}
        assert o["rs"] == [[0.0, 2.0], [4.0, 6.0]][r]
        assert o["async"] == [1.5, 1.5, 1.5]
        assert o["p2p"] == ([30.0, 40.0] if r == 0 else [3.0, 4.0])
        assert o["ip2p"] == [float(1 - r)]
        assert o["eng_rank"] == (r, world, True)
        assert o["err"] < 1e-12, o["err"]
        assert o["health"]


def test_mock_and_factory():
    from tneq_qc_amd.distributed import DistributedEngineSiamese, MockCommTorch, ReduceOp, get_comm_backend
    from tneq_qc_amd.distributed.comm import detect_best_backend
    m = get_comm_backend("mock", rank=0, world_size=1)
    assert isinstance(m, MockCommTorch) and m.rank == 0 and m.world_size == 1 and not m.is_initialized()
    t = torch.tensor([1.0, 2.0])
    assert torch.equal(m.allreduce(t, ReduceOp.AVG), t) and m.allgather(t)[0] is not t
    assert m.get_context().is_main_process
    assert detect_best_backend() == "mock"
    assert isinstance(get_comm_backend("auto"), MockCommTorch)
    with pytest.raises(ValueError):
        get_comm_backend("mpi")
    with pytest.raises(ValueError):
        get_comm_backend("carrier-pigeon")
    # the engine on a mock communicator and with none (the reference's `comm or get_comm_backend`)
    for comm in (m, None):
        eng = DistributedEngineSiamese(executor=_torch_executor, comm=comm)
        assert (eng.rank, eng.world_size) == (0, 1) and eng.group is None
        from oracle.greedy_ref import greedy_contract
        g, qr, qc, cores, states, mx = _setup()
        qc.cores_weights = {c: torch.tensor(cores[c]) for c in qc.cores}
        eng.init_distributed(qc)
        res = eng.contract_distributed([torch.tensor(s) for s in states], [torch.tensor(x) for x in mx])
        ref = np.abs(greedy_contract(qr, cores, states, mx)) ** 2
        assert np.abs(res.numpy() - ref).max() / np.abs(ref).max() < 1e-12
    # a mock runs no collectives, so a multi-rank mock is refused up front
    with pytest.raises(ValueError, match="runs no collectives"):
        DistributedEngineSiamese(executor=_torch_executor, comm=MockCommTorch(rank=0, world_size=4))


def test_failed_multirank_init_does_not_fall_back_to_a_mock(monkeypatch):
    """A launcher set WORLD_SIZE > 1 but the process group cannot be set up: the factory raises
    instead of returning a mock whose collectives are no-ops."""
    from tneq_qc_amd.distributed import get_comm_backend
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29999")
    with pytest.raises(RuntimeError, match="world size 2"):   # an unknown rendezvous scheme fails at once
        get_comm_backend("torch", torch_backend="gloo", init_method="nosuchscheme://x", world_size=2, rank=0)
