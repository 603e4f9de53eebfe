"""DistributedEngineSiamese drop-in (distributed/engine.py) on CPU: gloo groups of 2 and 3
ranks, the per-rank contractions injected as a differentiable torch executor (the GPU suite runs
the same engine on the native plan).  Checked against the oracle's literal GreedyStrategy
restatement (oracle/greedy_ref.py, the single-process sandwich) and torch autograd:
  * contract_distributed == |greedy sandwich|^2 on every rank (complex cores, batched Mx);
  * contract_distributed_with_gradient: the loss equals the single-process cross-entropy and a
    rank's gradients equal W x the single-process gradients of its own cores (the reference's
    AllReduceGrad / SendRecvGrad adjoints with the same loss on every rank);
  * TNTensor cores: the scales travel as log-scales; the value is unchanged;
  * the reference's partition rule and plan (distributed_engine.py:368-595)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_tree_cpu import _torch_executor


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    from oracle.qctn_ref import QCTNRef, random_cores
    from tneq_qc_amd.circuits import build_brick_wall_IM, incidence_to_graph
    from tneq_qc_amd.core import QCTN
    g = incidence_to_graph(build_brick_wall_IM(4, 2))
    qr = QCTNRef(g)
    cores = random_cores(qr, 11)
    q = QCTN(g)
    rng = np.random.default_rng(3)
    B = 3
    states = [np.array([1.0, 0.0], complex) for _ in range(q.nqubits)]
    mx = [rng.standard_normal((B, 2, 2)) + 1j * rng.standard_normal((B, 2, 2)) for _ in range(q.nqubits)]
    mx = [m + np.conj(np.swapaxes(m, 1, 2)) for m in mx]          # Hermitian measurements
    return g, qr, q, cores, states, mx


def _single_loss_and_grads(q, cores, states, mx):
    """Single process: the flat greedy einsum in torch + the reference's cross-entropy loss."""
    from tneq_qc_amd.contractor.greedy_symbolic import greedy_equation
    eq, recipe = greedy_equation(q, {i: 2 for i in range(q.nqubits)},
                                 {i: (3, 2, 2) for i in range(q.nqubits)},
                                 {c: cores[c].ndim for c in q.cores})
    ts = {c: torch.tensor(cores[c], requires_grad=True) for c in q.cores}
    ops = []
    for kind, k in recipe:
        if kind == "L":
            ops.append(ts[k])
        elif kind == "R":
            ops.append(ts[k].conj())
        elif kind == "S":
            ops.append(torch.tensor(states[k]))
        else:
            ops.append(torch.tensor(mx[k]))
    p = torch.einsum(eq, *ops).abs() ** 2
    loss = -torch.mean(torch.log(torch.clamp(p, min=1e-10)))
    g = torch.autograd.grad(loss, [ts[c] for c in q.cores])
    return float(loss), dict(zip(q.cores, g))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.greedy_ref import greedy_contract
        from tneq_qc_amd.core import TNTensor
        from tneq_qc_amd.distributed import DistributedEngineSiamese
        g, qr, qc, cores, states, mx = _setup()
        eng = DistributedEngineSiamese(executor=_torch_executor)
        qc.cores_weights = {c: torch.tensor(cores[c]) for c in qc.cores}
        plan = eng.init_distributed(qc)
        T = lambda a: torch.tensor(a)
        res = eng.contract_distributed([T(s) for s in states], [T(m) for m in mx])
        ref = np.abs(greedy_contract(qr, cores, states, mx)) ** 2
        err_fwd = float(np.abs(res.numpy() - ref).max() / np.abs(ref).max())
        loss, grads = eng.contract_distributed_with_gradient([T(s) for s in states], [T(m) for m in mx])
        ref_loss, ref_g = _single_loss_and_grads(qc, cores, states, mx)
        err_loss = abs(float(loss) - ref_loss) / abs(ref_loss)
        err_g = max(float((gr - world * ref_g[c]).abs().max() / ref_g[c].abs().max())
                    for c, gr in zip(eng._local_qctn.cores, grads))
        # TNTensor cores
        scales = {c: 2.0 ** (5 * (i % 4) - 7) for i, c in enumerate(qc.cores)}
        qc.cores_weights = {c: TNTensor(torch.tensor(cores[c] / scales[c]), scales[c]) for c in qc.cores}
        eng.init_distributed(qc)
        with torch.no_grad():
            r2 = eng.contract_distributed([T(s) for s in states], [T(m) for m in mx])
        val = r2.tensor.numpy() * r2.scale
        # the Born rule is applied to the raw sandwich; its scale is the product of the uses
        # (EngineSiamese.contract_with_compiled_strategy(ret_type='TNTensor') semantics)
        prod = float(np.prod([scales[c] ** 2 for c in qc.cores]))
        ref_tn = np.abs(greedy_contract(qr, {c: cores[c] / scales[c] for c in qc.cores}, states, mx)) ** 2 * prod
        err_tn = float(np.abs(val - ref_tn).max() / np.abs(ref_tn).max())
        q.put((rank, err_fwd, err_loss, err_g, err_tn, isinstance(r2, TNTensor), plan.num_stages,
               plan.local_cores, len(plan.inter_node_graph["cross_edges"])))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_engine_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = sorted(q.get(timeout=5) for _ in range(world))
    _, _, qc, _, _, _ = _setup()
    n = len(qc.cores)
    base, rem = divmod(n, world)
    idx = 0
    for rank, err_fwd, err_loss, err_g, err_tn, is_tn, stages, local, n_cross in got:
        assert err_fwd < 1e-12, (rank, err_fwd)
        assert err_loss < 1e-12, (rank, err_loss)
        assert err_g < 1e-10, (rank, err_g)
        assert err_tn < 1e-12 and is_tn, (rank, err_tn)
        assert stages == 1 + {2: 1, 3: 2}[world]
        size = base + (1 if rank < rem else 0)
        assert local == qc.cores[idx:idx + size]        # distributed_engine.py:439-452
        idx += size
        assert n_cross > 0


def test_world_one_needs_no_process_group():
    """the reference requires an initialised group even at world 1."""
    from oracle.greedy_ref import greedy_contract
    from tneq_qc_amd.distributed import DistributedEngineSiamese
    g, qr, qc, cores, states, mx = _setup()
    eng = DistributedEngineSiamese(executor=_torch_executor)
    qc.cores_weights = {c: torch.tensor(cores[c]) for c in qc.cores}
    plan = eng.init_distributed(qc)
    assert plan.num_stages == 1 and plan.local_cores == qc.cores
    res = eng.contract_distributed([torch.tensor(s) for s in states], [torch.tensor(m) for m in mx])
    ref = np.abs(greedy_contract(qr, cores, states, mx)) ** 2
    assert np.abs(res.numpy() - ref).max() / np.abs(ref).max() < 1e-12
