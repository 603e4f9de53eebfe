"""SGDG on the HIP kernel (tq_sgdg_step via tneq_qc_amd.optim.SGDG) vs the oracle's restatement
of stiefel_optimizer_complex.py:77-176, several steps with momentum, for the workload's 4x4
complex cores (Stiefel / Cayley branch, incl. the random qr_retraction draw) and a rows > cols
parameter (SGD branch with weight decay / nesterov).  Same Python `random` seed on both sides.
Tolerances: complex128 / float64 1e-12, complex64 / float32 1e-5 (relative to max |p|)."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = {"complex128": 1e-12, "float64": 1e-12, "complex64": 1e-5, "float32": 1e-5}


def _params(rng, dtype, cplx):
    shapes = [(2, 2, 2, 2)] * 5 + [(2, 2, 2)] + [(4, 2)]
    out = []
    for s in shapes:
        a = rng.standard_normal(s)
        if cplx:
            a = a + 1j * rng.standard_normal(s)
        out.append(a.astype(dtype))
    return out


@pytest.mark.parametrize("dtype", ["complex128", "complex64", "float64", "float32"])
def test_sgdg_steps_match_oracle(dev, dtype):
    import torch
    from oracle.optim_ref import sgdg_step
    from tneq_qc_amd.optim import SGDG
    cplx = dtype.startswith("complex")
    rng = np.random.default_rng(7)
    ref = _params(rng, np.dtype(dtype), cplx)
    params = [torch.nn.Parameter(torch.from_numpy(p.copy()).to(dev)) for p in ref]
    hp = dict(lr=0.05, momentum=0.9, weight_decay=0.01, nesterov=False, stiefel=True)
    opt = SGDG(params, **hp)
    state = {}
    seeds = [next(s for s in range(10000) if (random.seed(s), random.randint(1, 101))[1] == 1), 5, 6]
    for step, seed in enumerate(seeds):
        grads = [(rng.standard_normal(p.shape) + (1j * rng.standard_normal(p.shape) if cplx else 0)).astype(dtype)
                 for p in ref]
        for p, g in zip(params, grads):
            p.grad = torch.from_numpy(g.copy()).to(dev)
        random.seed(seed)
        opt.step()
        random.seed(seed)
        sgdg_step(ref, [g.copy() for g in grads], state, **hp)
        torch.cuda.synchronize()
        for i, (p, r) in enumerate(zip(params, ref)):
            got = p.detach().cpu().numpy()
            err = np.abs(got - r).max() / max(np.abs(r).max(), 1e-30)
            assert err < TOL[dtype], (step, i, err)
            if "momentum_buffer" in state.get(i, {}):
                b = opt.state[p]["momentum_buffer"].cpu().numpy()
                rb = state[i]["momentum_buffer"]
                assert np.abs(b - rb).max() / max(np.abs(rb).max(), 1e-30) < TOL[dtype] * 10, (step, i)


def test_sgdg_workload_loop_keeps_cores_unitary_and_fits(dev):
    """A few iterations of the symmetry-breaking fit (symmetry_breaking_quantum.py:203-230):
    fidelity loss through the HIP expression, backward, HIP SGDG step; cores stay unitary and
    the loss decreases."""
    import torch
    from tneq_qc_amd.circuits import BrickWall
    from tneq_qc_amd.contractor import EinsumStrategy
    from tneq_qc_amd.optim import SGDG
    bw = BrickWall(4, 4, 3)
    q = bw.qctn
    eq, shapes = EinsumStrategy.build_core_only_expression(q)
    expr = EinsumStrategy.create_contract_expression(eq, shapes)
    tgt = expr(*[torch.from_numpy(bw.cores[c]).to(dev) for c in q.cores]).detach().reshape(-1)
    rng = np.random.default_rng(0)
    init = []
    for c in q.cores:
        a, r = np.linalg.qr(rng.standard_normal((4, 4)) + 1j * rng.standard_normal((4, 4)))
        init.append((a * (np.diag(r) / np.abs(np.diag(r)))[None, :]).reshape(2, 2, 2, 2))
    params = [torch.nn.Parameter(torch.from_numpy(a).to(dev)) for a in init]
    opt = SGDG(params, lr=1e-2, stiefel=True, momentum=0.9)
    losses = []
    random.seed(0)
    for _ in range(30):
        opt.zero_grad()
        out = expr(*params).reshape(-1)
        num = torch.vdot(tgt, out).abs() ** 2
        den = (torch.vdot(tgt, tgt).real * torch.vdot(out, out).real).clamp_min(1e-12)
        loss = 1.0 - num / den
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]
    eye = torch.eye(4, dtype=torch.complex128, device=dev)
    for p in params:
        u = p.detach().reshape(4, 4)
        assert torch.allclose(u @ u.conj().T, eye, atol=1e-10)


@pytest.mark.parametrize("dtype", ["complex128", "complex64", "float64"])
def test_sgdg_large_and_1d_stiefel_params_match_oracle(dev, dtype):
    """Stiefel parameters beyond the LDS-resident size: a 1-D parameter (1 x 100), a
    bond-dimension-3 core (3,3,3,3) -> 9 x 9 (LDS), a (4,4,4,4) core -> 16 x 16, a (2,40) -> 2 x 40
    and a (3, 64) -> 3 x 64 parameter (global scratch), with momentum and a forced qr_retraction,
    against the oracle over 3 steps."""
    import torch
    from oracle.optim_ref import sgdg_step
    from tneq_qc_amd.optim import SGDG
    cplx = dtype.startswith("complex")
    rng = np.random.default_rng(11)
    shapes = [(100,), (3, 3, 3, 3), (4, 4, 4, 4), (2, 40), (3, 64)]
    ref = []
    for s in shapes:
        a = rng.standard_normal(s) + (1j * rng.standard_normal(s) if cplx else 0)
        ref.append(a.astype(dtype))
    params = [torch.nn.Parameter(torch.from_numpy(p.copy()).to(dev)) for p in ref]
    hp = dict(lr=0.05, momentum=0.9, stiefel=True)
    opt = SGDG(params, **hp)
    state = {}
    seeds = [next(s for s in range(10000) if (random.seed(s), random.randint(1, 101))[1] == 1), 5, 6]
    for step, seed in enumerate(seeds):
        grads = [(rng.standard_normal(p.shape) + (1j * rng.standard_normal(p.shape) if cplx else 0)).astype(dtype)
                 for p in ref]
        for p, g in zip(params, grads):
            p.grad = torch.from_numpy(g.copy()).to(dev)
        random.seed(seed)
        opt.step()
        random.seed(seed)
        sgdg_step(ref, [g.copy() for g in grads], state, **hp)
        torch.cuda.synchronize()
        for i, (p, r) in enumerate(zip(params, ref)):
            got = p.detach().cpu().numpy()
            err = np.abs(got - r).max() / max(np.abs(r).max(), 1e-30)
            assert err < TOL[dtype] * 10, (step, shapes[i], err)


def test_sgdg_rejects_oversized_before_touching_anything(dev):
    """A Stiefel parameter over the column limit raises before any random draw, momentum buffer
    or launch: the other parameters, the optimizer state and `random`'s stream are unchanged."""
    import torch
    from tneq_qc_amd.optim import SGDG
    from tneq_qc_amd.optim.stiefel_optimizer_complex import MAX_STIEFEL_COLS
    ok = torch.nn.Parameter(torch.randn(2, 2, 2, 2, dtype=torch.complex128, device=dev))
    big = torch.nn.Parameter(torch.randn(MAX_STIEFEL_COLS + 1, dtype=torch.complex128, device=dev))
    for p in (ok, big):
        p.grad = torch.randn_like(p)
    before = ok.detach().clone()
    opt = SGDG([ok, big], lr=0.1, momentum=0.9, stiefel=True)
    random.seed(3)
    with pytest.raises(ValueError):
        opt.step()
    assert random.randint(1, 101) == (random.seed(3), random.randint(1, 101))[1]
    assert torch.equal(ok.detach(), before)
    assert len(opt.state) == 0


@pytest.mark.parametrize("dtype", ["complex128", "complex64"])
def test_sgdg_wide_params_low_rank_timed(dev, dtype):
    """wide Stiefel parameters on the global scratch.  A 1 x 2048 (1-D) and a 9 x 64
    parameter take the low-rank (Woodbury) form (W has rank <= 2 rows < cols: O(cols^2 rows)
    work, O(cols rows) scratch), a 40 x 64 one the dense Gauss-Jordan; all against the oracle
    over 2 steps with momentum, and the 1 x 2048 step timed (the dense form took seconds)."""
    import time
    import torch
    from oracle.optim_ref import sgdg_step
    from tneq_qc_amd.optim import SGDG
    rng = np.random.default_rng(5)
    shapes = [(2048,), (9, 64), (40, 64)]
    ref = [(rng.standard_normal(s) + 1j * rng.standard_normal(s)).astype(dtype) for s in shapes]
    params = [torch.nn.Parameter(torch.from_numpy(p.copy()).to(dev)) for p in ref]
    hp = dict(lr=0.05, momentum=0.9, stiefel=True)
    opt = SGDG(params, **hp)
    state = {}
    for step, seed in enumerate([5, 6]):
        grads = [(rng.standard_normal(p.shape) + 1j * rng.standard_normal(p.shape)).astype(dtype) for p in ref]
        for p, g in zip(params, grads):
            p.grad = torch.from_numpy(g.copy()).to(dev)
        random.seed(seed)
        opt.step()
        random.seed(seed)
        sgdg_step(ref, [g.copy() for g in grads], state, **hp)
        torch.cuda.synchronize()
        for i, (p, r) in enumerate(zip(params, ref)):
            err = np.abs(p.detach().cpu().numpy() - r).max() / np.abs(r).max()
            assert err < TOL[dtype] * 10, (step, shapes[i], err)
            b = opt.state[p]["momentum_buffer"].cpu().numpy()
            rb = state[i]["momentum_buffer"]
            assert np.abs(b - rb).max() / max(np.abs(rb).max(), 1e-30) < TOL[dtype] * 100, (step, shapes[i])
    wide = SGDG([params[0]], **hp)
    random.seed(5)
    wide.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        wide.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 5 * 1e3
    print(f"SGDG 1 x 2048 {dtype}: {ms:.3f} ms per step")
    assert ms < 50.0, ms


@pytest.mark.parametrize("dtype", ["complex128", "float64"])
def test_sgdg_cached_steady_state_matches_oracle(dev, dtype):
    """The steady-state path (SGDG caches a group's checks and launch arrays while the
    parameters, gradients and buffers stay the same tensors -- a training loop whose backward
    writes the same .grad tensors, e.g. a replayed hipGraph): gradients updated IN PLACE over
    4 steps match the oracle; then one gradient tensor is replaced (cache miss: the full path)
    and the state is reset (a new buffer: miss again), still matching.  The retraction draws
    come from an rng= generator, the oracle draws from an equal one."""
    import torch
    from oracle.optim_ref import sgdg_step
    from tneq_qc_amd.optim import SGDG
    cplx = dtype.startswith("complex")
    rng = np.random.default_rng(11)
    ref = _params(rng, np.dtype(dtype), cplx)
    params = [torch.nn.Parameter(torch.from_numpy(p.copy()).to(dev)) for p in ref]
    hp = dict(lr=0.05, momentum=0.9, weight_decay=0.01, nesterov=False, stiefel=True)
    # a seed whose first draw retracts
    seed = next(s for s in range(10000) if random.Random(s).randint(1, 101) == 1)
    opt = SGDG(params, rng=random.Random(seed), **hp)
    ref_rng = random.Random(seed)
    state = {}
    for p in params:
        p.grad = torch.zeros_like(p)
    for step in range(7):
        grads = [(rng.standard_normal(p.shape) + (1j * rng.standard_normal(p.shape) if cplx else 0)).astype(dtype)
                 for p in ref]
        if step == 4:        # a new gradient tensor for one parameter: the cache misses
            params[2].grad = torch.empty_like(params[2])
        if step == 5:        # the optimizer state reset: new buffers, a miss again
            opt.state.clear()
            state.clear()
        for p, g in zip(params, grads):
            p.grad.copy_(torch.from_numpy(g.copy()))   # in place: the same .grad tensors
        opt.step()
        sgdg_step(ref, [g.copy() for g in grads], state, rng=ref_rng, **hp)
        torch.cuda.synchronize()
        for i, (p, r) in enumerate(zip(params, ref)):
            err = np.abs(p.detach().cpu().numpy() - r).max() / max(np.abs(r).max(), 1e-30)
            assert err < TOL[dtype], (step, i, err)
    assert 0 in getattr(opt, "_sgdg_cache", {})   # the steady state was cached
