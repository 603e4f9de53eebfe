"""The benchmarked C5 training step (bench.py's `c5_train` line = scripts/c5_bench.py) pinned
against an independent host computation at FULL C5 size.

GPU side, exactly as the bench runs it: the 8 pruning candidates of c5_bench.setup (34-core
split/merge core-only forward to 2^16 amplitudes, complex128), forward + fidelity loss + backward
captured once per candidate as a hipGraph (graphs.capture_step), each candidate on its own
stream, SGDG (`tq_sgdg_step`) eager with the candidate's own retraction-draw stream; 3 steps.

Host side (the reference's math, symmetry_breaking_quantum.py:196-238 and
stiefel_optimizer_complex.py:77-176): the target by the oracle's numpy pairwise executor
(oracle/contract_ref.py), every candidate's forward as pairwise torch.tensordot on the CPU (what
opt_einsum's ContractExpression runs), torch autograd for the gradients, and the oracle SGDG
(oracle/optim_ref.py) drawing from random.Random(1000 + k) -- the stream c5_bench gives
candidate k.

Compared: the target, every loss of all 3 steps, every gradient of step 1 and every parameter
after each step.  Tolerance 1e-10 relative (complex128)."""
import importlib.util
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 1e-10
STEPS = 3


def _c5():
    spec = importlib.util.spec_from_file_location("c5_bench", os.path.join(ROOT, "scripts", "c5_bench.py"))
    cb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cb)
    return cb


def _close(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    scale = max(1.0, float(np.abs(b).max()))
    err = float(np.abs(a - b).max())
    assert err <= TOL * scale, f"{what}: max |diff| {err:.3e} (scale {scale:.3e})"


def test_c5_training_step_matches_host_reference(dev):
    import torch
    from oracle.contract_ref import contract
    from tneq_qc_amd.circuits import BrickWall, TRAIN_MASK
    from tneq_qc_amd.contractor import EinsumStrategy
    cb = _c5()
    target, cands = cb.setup(dev)
    assert len(cands) == len(cb.CANDIDATES) == 8
    assert all(len(c[1]) == 34 for c in cands)

    # --- host side: independent target, initial parameters copied before any GPU step ---
    tgt_bw = BrickWall(cb.N_Q, cb.DEPTH, seed=5, mask=TRAIN_MASK)
    eq_t, _ = EinsumStrategy.build_core_only_expression(tgt_bw.qctn)
    tgt_np = contract(eq_t, *[tgt_bw.cores[c] for c in tgt_bw.qctn.cores]).reshape(-1)
    _close(target.cpu().numpy(), tgt_np, "target amplitudes")
    host = [([p.detach().cpu().numpy().copy() for p in c[1]], {}, random.Random(1000 + k))
            for k, c in enumerate(cands)]

    # --- GPU side: the bench's graphed, multi-stream step ---
    streams = [torch.cuda.Stream(dev) for _ in cands]
    graphs = cb.capture(target, cands, dev)
    gpu_losses, gpu_params, gpu_grads = [], [], None
    for s in range(STEPS):
        losses = cb.gpu_step(target, cands, streams, graphs)
        torch.cuda.synchronize()
        gpu_losses.append([float(l.detach()) for l in losses])
        gpu_params.append([[p.detach().cpu().numpy() for p in c[1]] for c in cands])
        if s == 0:
            gpu_grads = [[p.grad.detach().cpu().numpy() for p in c[1]] for c in cands]

    tgt = torch.from_numpy(tgt_np)
    for s in range(STEPS):
        for k, (expr, _, _, _, _, _) in enumerate(cands):
            ps, state, rng = host[k]
            loss, grads = cb.cpu_train_step(expr, ps, state, tgt, rng=rng)
            assert abs(gpu_losses[s][k] - loss) <= TOL * max(1.0, abs(loss)), (s, k, gpu_losses[s][k], loss)
            if s == 0:
                for i, (g_gpu, g_cpu) in enumerate(zip(gpu_grads[k], grads)):
                    _close(g_gpu, g_cpu, f"step 1 candidate {k} gradient {i}")
            for i, (p_gpu, p_cpu) in enumerate(zip(gpu_params[s][k], ps)):
                _close(p_gpu, p_cpu, f"step {s + 1} candidate {k} parameter {i}")
    # the fits move: the losses change over the steps
    assert any(abs(gpu_losses[-1][k] - gpu_losses[0][k]) > 1e-9 for k in range(len(cands)))
