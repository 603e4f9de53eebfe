"""Reverse-mode autograd through the HIP expression's pairwise path (expression._ReverseTree)
vs torch.einsum autograd on the CPU (complex128 / float64 reference): random networks with
batch modes, single-side sums and broadcast-back gradients, mixed real / complex operands,
partial requires_grad, and the symmetry-breaking fidelity loss (symmetry_breaking_quantum.py:
203-224) on a 5-qubit brick wall (torch.einsum, the CPU reference here, takes <= 52 symbols; the
full 8-qubit C5 ansatz is pinned in tests/test_c5_parity_gpu.py against pairwise tensordot).
Tolerance 1e-10 (float64 / complex128)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(eq, shapes, dtypes, req, seed=0):
    import torch
    from tneq_qc_amd.expression import HipContractExpression
    rng = np.random.default_rng(seed)
    arrs = []
    for s, dt in zip(shapes, dtypes):
        a = rng.standard_normal(s)
        if dt == "c":
            a = a + 1j * rng.standard_normal(s)
        arrs.append(a)
    ref = [torch.tensor(a, requires_grad=r) for a, r in zip(arrs, req)]
    cplx = any(np.iscomplexobj(a) for a in arrs)
    # torch.einsum wants one dtype: promote inside the graph (the cast is differentiable)
    out_r = torch.einsum(eq, *[t.to(torch.complex128) if cplx else t for t in ref])
    w = torch.tensor(rng.standard_normal(out_r.shape) + (1j * rng.standard_normal(out_r.shape) if out_r.is_complex() else 0))
    loss_r = (out_r * w).real.sum() if out_r.is_complex() else (out_r * w).sum()
    gr = torch.autograd.grad(loss_r, [t for t, r in zip(ref, req) if r])
    ts = [torch.tensor(a, device="cuda", requires_grad=r) for a, r in zip(arrs, req)]
    e = HipContractExpression(eq, *shapes)
    out = e(*ts)
    assert torch.allclose(out.cpu(), out_r.detach(), atol=1e-11)
    wd = w.to("cuda")
    loss = (out * wd).real.sum() if out.is_complex() else (out * wd).sum()
    g = torch.autograd.grad(loss, [t for t, r in zip(ts, req) if r])
    for a, b in zip(g, gr):
        assert a.shape == b.shape and a.dtype == b.dtype
        assert torch.allclose(a.cpu(), b, atol=1e-10), (a.cpu() - b).abs().max()


@pytest.mark.parametrize("case", range(6))
def test_reverse_mode_matches_torch_autograd(dev, case):
    cases = [
        ("ab,bc,cd->ad", [(3, 4), (4, 5), (5, 2)], "ccc", [1, 1, 1]),
        ("abx,bcy,cd->ady", [(3, 4, 2), (4, 5, 3), (5, 2)], "crc", [1, 1, 0]),   # x summed on one side
        ("zab,zbc->zac", [(2, 3, 4), (2, 4, 3)], "cc", [1, 1]),                 # batch mode
        ("ab,bc,ca->", [(3, 4), (4, 5), (5, 3)], "rrr", [1, 0, 1]),             # scalar out
        ("ijkl,klmn,mnop,opij->ikmo", [(2,) * 4] * 4, "cccc", [1, 1, 1, 1]),
        ("ab->ba", [(3, 4)], "c", [1]),                                         # one operand
    ]
    eq, shapes, dts, req = cases[case]
    _check(eq, shapes, dts, [bool(r) for r in req], seed=case)


def test_fidelity_loss_gradients_on_a_brick_wall(dev):
    import torch
    from tneq_qc_amd.circuits import BrickWall
    from tneq_qc_amd.contractor import EinsumStrategy
    bw = BrickWall(5, 4, 9)   # torch.einsum (the CPU reference) takes <= 52 symbols
    q = bw.qctn
    eq, shapes = EinsumStrategy.build_core_only_expression(q)
    expr = EinsumStrategy.create_contract_expression(eq, shapes, optimize="auto")
    rng = np.random.default_rng(3)
    tgt_np = rng.standard_normal(expr.out_shape) + 1j * rng.standard_normal(expr.out_shape)
    def loss_of(params, tgt):
        if params[0].is_cuda:
            out = expr(*params).reshape(-1)
        else:
            out = torch.einsum(eq, *params).reshape(-1)
        num = torch.vdot(tgt, out).abs() ** 2
        den = (torch.vdot(tgt, tgt).real * torch.vdot(out, out).real).clamp_min(1e-12)
        return 1.0 - num / den
    pc = [torch.tensor(bw.cores[c], requires_grad=True) for c in q.cores]
    lc = loss_of(pc, torch.tensor(tgt_np).reshape(-1))
    gc = torch.autograd.grad(lc, pc)
    pg = [torch.tensor(bw.cores[c], device="cuda", requires_grad=True) for c in q.cores]
    lg = loss_of(pg, torch.tensor(tgt_np, device="cuda").reshape(-1))
    gg = torch.autograd.grad(lg, pg)
    assert abs(lg.item() - lc.item()) < 1e-12
    for a, b in zip(gg, gc):
        assert torch.allclose(a.cpu(), b, atol=1e-10)


def test_repeated_steps_hit_the_captured_graph_and_stay_exact(dev):
    """Training-loop shape: same parameter tensors updated in place, loss/backward repeated —
    the forward / backward launch sequences are captured once and replayed; a second forward
    before the first backward forces a recompute (static buffers are shared)."""
    import torch
    from tneq_qc_amd.circuits import BrickWall
    from tneq_qc_amd.contractor import EinsumStrategy
    bw = BrickWall(5, 4, 2)
    q = bw.qctn
    eq, shapes = EinsumStrategy.build_core_only_expression(q)
    expr = EinsumStrategy.create_contract_expression(eq, shapes)
    pg = [torch.nn.Parameter(torch.tensor(bw.cores[c], device="cuda")) for c in q.cores]
    pc = [torch.tensor(bw.cores[c], requires_grad=True) for c in q.cores]
    for it in range(4):
        lg = expr(*pg).abs().square().sum()
        lc = torch.einsum(eq, *pc).abs().square().sum()
        gg = torch.autograd.grad(lg, pg)
        gc = torch.autograd.grad(lc, pc)
        for a, b in zip(gg, gc):
            assert torch.allclose(a.cpu(), b, atol=1e-10), it
        with torch.no_grad():
            for p_, c_, a_ in zip(pg, pc, gc):
                p_.mul_(0.9).add_(0.01 * a_.to("cuda"))
                c_.mul_(0.9).add_(0.01 * a_)
    rt = expr.reverse_tree(torch.complex128).runtime(torch.complex128, pg[0].device)
    assert len(rt.graphs) >= 2       # forward and backward captured
    # two forwards, then the first backward: recomputed from its own inputs
    x1 = [p.detach().clone().requires_grad_(True) for p in pg]
    x2 = [p.detach().mul(1.1).requires_grad_(True) for p in pg]
    l1 = expr(*x1).abs().square().sum()
    l2 = expr(*x2).abs().square().sum()
    g1 = torch.autograd.grad(l1, x1)
    c1 = [p.detach().cpu().clone().requires_grad_(True) for p in pg]
    r1 = torch.autograd.grad(torch.einsum(eq, *c1).abs().square().sum(), c1)
    for a, b in zip(g1, r1):
        assert torch.allclose(a.cpu(), b, atol=1e-10)


def test_retain_graph_second_backward_and_inplace_guard(dev):
    """a second backward with retain_graph=True gives the same gradients; an in-place
    change of an input between forward and backward raises (autograd's version counter), as
    torch.einsum's own backward would."""
    import torch
    from tneq_qc_amd.expression import HipContractExpression
    rng = np.random.default_rng(3)
    shapes = [(3, 4), (4, 5), (5, 3)]
    ts = [torch.tensor(rng.standard_normal(s) + 1j * rng.standard_normal(s), device=dev, requires_grad=True)
          for s in shapes]
    e = HipContractExpression("ab,bc,ca->", *shapes)
    out = e(*ts)
    loss = (out * (2 - 1j)).real
    g1 = torch.autograd.grad(loss, ts, retain_graph=True)
    g2 = torch.autograd.grad(loss, ts)
    for a, b in zip(g1, g2):
        assert torch.allclose(a, b, atol=1e-12)
    x = [t.detach().clone().requires_grad_(True) for t in ts]
    y = [t * 1 for t in x]   # non-leaf inputs that can be modified in place
    out = e(*y)
    with torch.no_grad():
        y[1].mul_(2.0)
    with pytest.raises(RuntimeError):
        out.real.backward()


def test_one_expression_on_two_streams(dev):
    """one expression differentiated concurrently on two streams keeps per-stream
    static buffers: both gradients equal the single-stream ones."""
    import torch
    from tneq_qc_amd.expression import HipContractExpression
    rng = np.random.default_rng(4)
    shapes = [(8, 8, 4), (4, 8), (8, 8)]
    e = HipContractExpression("abc,cd,db->a", *shapes)
    sets = [[torch.tensor(rng.standard_normal(s) + 1j * rng.standard_normal(s), device=dev, requires_grad=True)
             for s in shapes] for _ in range(2)]
    ref = []
    for ts in sets:
        ref.append(torch.autograd.grad(e(*ts).abs().sum(), ts))
    st = [torch.cuda.Stream(dev) for _ in range(2)]
    got = [None, None]
    for _ in range(3):   # the third round replays captured graphs
        cur = torch.cuda.current_stream(dev)
        for k in range(2):
            st[k].wait_stream(cur)
            with torch.cuda.stream(st[k]):
                got[k] = torch.autograd.grad(e(*sets[k]).abs().sum(), sets[k])
        for k in range(2):
            cur.wait_stream(st[k])
        torch.cuda.synchronize(dev)
        for k in range(2):
            for a, b in zip(got[k], ref[k]):
                assert torch.allclose(a, b, atol=1e-11)
