"""HIP kernel parity on the GPU: permute (bit-exact), MFMA GEMM and pairwise contraction
(tolerance vs a float64/complex128 numpy product of the same operands)."""
import itertools

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DTYPES = ["float32", "float64", "complex64", "complex128"]
# relative tolerance (max error / max |exact|) vs an exact (f64/c128) reference: the north-star
# amplitude tolerances (complex64 2e-5, complex128 1e-12), fixed — not scaled with K
TOL = {"float32": 2e-5, "complex64": 2e-5, "float64": 1e-12, "complex128": 1e-12}


def _rand(rng, shape, dt):
    x = rng.standard_normal(shape)
    if dt.startswith("complex"):
        x = x + 1j * rng.standard_normal(shape)
    return x.astype(dt)


@pytest.fixture(scope="module")
def T(dev):
    import torch
    import tneq_qc_amd.ops as ops  # noqa: F401
    return torch


def _to(T, dev, a):
    return T.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("dt", DTYPES)
def test_permute_binary_legs(T, dev, dt):
    import tneq_qc_amd.ops as ops
    rng = np.random.default_rng(1)
    for rank in (1, 3, 7, 12, 16, 20):
        x = _rand(rng, (2,) * rank, dt)
        xd = _to(T, dev, x)
        for _ in range(4):
            p = rng.permutation(rank)
            y = ops.permute(xd, list(p)).cpu().numpy()
            assert np.array_equal(y, np.transpose(x, p)), (rank, p)


@pytest.mark.parametrize("dt", ["complex64", "float64"])
def test_permute_mixed_extents_and_views(T, dev, dt):
    import tneq_qc_amd.ops as ops
    rng = np.random.default_rng(2)
    shapes = [(3, 5, 7), (64, 33), (1, 4, 1, 9, 2), (128, 2, 2, 130), (5,), (1,), (17, 1, 4096)]
    for s in shapes:
        x = _rand(rng, s, dt)
        xd = _to(T, dev, x)
        for p in list(itertools.permutations(range(len(s))))[:6]:
            y = ops.permute(xd, p).cpu().numpy()
            assert np.array_equal(y, np.transpose(x, p)), (s, p)
    # a sliced (strided) view: fix index 1 of the middle leg
    x = _rand(rng, (2,) * 14, dt)
    xd = _to(T, dev, x)
    v = xd[:, :, 1]
    y = ops.permute(v, list(range(v.ndim))[::-1]).cpu().numpy()
    assert np.array_equal(y, np.transpose(x[:, :, 1], list(range(13))[::-1]))


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_shapes(T, dev, dt, ta, tb):
    import tneq_qc_amd.ops as ops
    rng = np.random.default_rng(3)
    exact = "complex128" if dt.startswith("complex") else "float64"
    for (M, N, K, B) in [(1, 1, 1, 1), (4, 4, 4, 3), (33, 65, 17, 2), (128, 128, 16, 1),
                         (200, 70, 300, 1), (64, 256, 4096, 1), (3, 300, 2, 5)]:
        a = _rand(rng, (B, K, M) if ta else (B, M, K), dt)
        b = _rand(rng, (B, N, K) if tb else (B, K, N), dt)
        c = ops.gemm(_to(T, dev, a), _to(T, dev, b), bool(ta), bool(tb)).cpu().numpy()
        ae = a.astype(exact)
        be = b.astype(exact)
        ref = np.matmul(np.swapaxes(ae, 1, 2) if ta else ae, np.swapaxes(be, 1, 2) if tb else be)
        err = np.abs(c - ref).max() / max(1e-30, np.abs(ref).max())
        assert err < TOL[dt], (M, N, K, B, err)


def test_gemm_beta_and_splitk(T, dev):
    import tneq_qc_amd.ops as ops
    rng = np.random.default_rng(4)
    a = _rand(rng, (256, 8192), "complex64")
    b = _rand(rng, (8192, 128), "complex64")
    c0 = _rand(rng, (1, 256, 128), "complex64")
    cd = _to(T, dev, c0)
    ops.gemm(_to(T, dev, a), _to(T, dev, b), out=cd, beta=1.0)
    ref = a.astype("complex128") @ b.astype("complex128") + c0[0]
    err = np.abs(cd.cpu().numpy()[0] - ref).max() / np.abs(ref).max()
    assert err < 1e-5


@pytest.mark.parametrize("dt", ["complex64", "complex128", "float32"])
def test_contract_pair_random(T, dev, dt):
    import tneq_qc_amd.ops as ops
    rng = np.random.default_rng(5)
    exact = "complex128" if dt.startswith("complex") else "float64"
    for trial in range(30):
        nmodes = rng.integers(2, 9)
        ext = {m: int(rng.integers(1, 4)) for m in range(nmodes)}
        ma = list(rng.choice(nmodes, size=rng.integers(1, nmodes + 1), replace=False))
        mb = list(rng.choice(nmodes, size=rng.integers(1, nmodes + 1), replace=False))
        allm = sorted(set(ma) | set(mb))
        mc = [m for m in allm if rng.random() < 0.5]
        rng.shuffle(mc)
        a = _rand(rng, [ext[m] for m in ma], dt)
        b = _rand(rng, [ext[m] for m in mb], dt)
        c = ops.contract_pair(ma, _to(T, dev, a), mb, _to(T, dev, b), mc).cpu().numpy()
        L = "abcdefghij"
        eq = "".join(L[m] for m in ma) + "," + "".join(L[m] for m in mb) + "->" + "".join(L[m] for m in mc)
        ref = np.einsum(eq, a.astype(exact), b.astype(exact))
        scale = max(1.0, np.abs(ref).max())
        tol = 1e-12 if dt == "complex128" else 1e-4
        assert np.abs(c - ref).max() / scale < tol, (eq, trial)


def test_contract_pair_gate_apply(T, dev):
    """(2,)*20 state absorbing a (2,2,2,2) gate on two adjacent legs -> the APPLY lowering."""
    import tneq_qc_amd.ops as ops
    rng = np.random.default_rng(6)
    s = _rand(rng, (2,) * 20, "complex64")
    g = _rand(rng, (2, 2, 2, 2), "complex64")
    ma = list(range(20))
    mg = [7, 8, 100, 101]
    mc = ma[:7] + [100, 101] + ma[9:]
    c = ops.contract_pair(ma, _to(T, dev, s), mg, _to(T, dev, g), mc).cpu().numpy()
    ref = np.moveaxis(np.tensordot(s.astype("complex128"), g.astype("complex128"), axes=([7, 8], [0, 1])),
                      [18, 19], [7, 8])
    assert np.abs(c - ref).max() / np.abs(ref).max() < 1e-5


@pytest.fixture(params=["f16", "f16w4", "f16g3", "f16r4", "f16s16", "f16g3w8", "f16g3o", "f16g3p", "f16g3s", "f16g3q", "bf16", "f32"])
def c64_kernel(request):
    """Runs a test once on each complex64 K-outer kernel: the f16 2-term split of the scaled
    operands (default tile; "f16w4": 4 waves of 64x64, "f16g3": the same with Gauss's 3M
    product, "f16r4": the default tile on a 4-slot LDS ring with one barrier per two K-steps,
    "f16s16": the default tile on v_mfma_f32_16x16x32_f16 (K-chunks of a multiple of 32; others
    fall back to the default kernel), "f16g3w8": the 64 x 32 tile with Gauss's 3M product, "f16g3o":
    the same with 3 staging sets and the ordered term pairs (the library default), "f16g3p":
    "f16g3w8" with product-major MFMA order, "f16g3s": product-major with the fragments read per
    product group and 3 staging sets, "f16g3q": "f16g3s" with the barrier before the last group
    and the next step's first group read under it — tq_library_set("gemm_f16_var", 1 / 2 / 3 / 4 /
    5 / 6 / 7 / 8 / 9)), the bf16
    3-term split kernel
    (tq_library_set("gemm_f16", 0)) and the f32-MFMA LDS-DMA kernel (tq_library_set("gemm_bf16",
    0)); restores the defaults."""
    import tneq_qc_amd._lib as _lib
    L = _lib.lib()
    keys = (b"gemm_bf16", b"gemm_f16", b"gemm_f16_var")
    before = [L.tq_library_query(k) for k in keys]
    p = request.param
    assert L.tq_library_set(b"gemm_bf16", 0 if p == "f32" else 1) == 0
    assert L.tq_library_set(b"gemm_f16", 1 if p.startswith("f16") else 0) == 0
    assert L.tq_library_set(b"gemm_f16_var", {"f16w4": 1, "f16g3": 2, "f16r4": 3, "f16s16": 4, "f16g3w8": 5, "f16g3o": 6, "f16g3p": 7, "f16g3s": 8, "f16g3q": 9}.get(p, 0)) == 0
    yield p
    for k, v in zip(keys, before):
        L.tq_library_set(k, v)


@pytest.mark.parametrize("M,N,K,B,beta", [(256, 128, 16, 1, 0.0), (256, 128, 48, 3, 0.0),
                                           (512, 256, 4096, 1, 1.0), (1024, 1024, 8192, 1, 0.0),
                                           (256, 256, 2048, 2, 0.5), (768, 384, 1024, 1, 0.0),
                                           (128, 128, 32, 1, 0.0), (384, 256, 80, 2, 1.0),
                                           (128, 128, 64, 1, 0.5), (256, 256, 96, 2, 0.0)])
def test_gemm_c64_kouter_fast_path(T, dev, c64_kernel, M, N, K, B, beta):
    """complex64 with A stored K x M and B stored K x N, on both fast kernels (bf16 3-term split:
    register-staged split into a double-buffered LDS image; f32 MFMA: LDS-DMA 3-stage ring) —
    shapes on the tile grid, batched, with beta, odd and even K-step counts (1, 2, 3, 5),
    single and multiple splits."""
    import tneq_qc_amd.ops as ops
    rng = np.random.default_rng(7)
    a = _rand(rng, (B, K, M), "complex64")
    b = _rand(rng, (B, K, N), "complex64")
    c0 = _rand(rng, (B, M, N), "complex64")
    cd = _to(T, dev, c0)
    ops.gemm(_to(T, dev, a), _to(T, dev, b), True, False, out=cd, beta=beta)
    ref = np.matmul(np.swapaxes(a.astype("complex128"), 1, 2), b.astype("complex128")) + beta * c0
    err = np.abs(cd.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err < TOL["complex64"], (M, N, K, B, err)


@pytest.mark.parametrize("sa,sb", [(1e-30, 1e25), (1e20, 1e-12), (2e-32, 1e-3), (1.0, 0.0), (7.0, 1e-3)])
def test_gemm_c64_split_operand_scales(T, dev, c64_kernel, sa, sb):
    """Operand magnitudes far from 1 (the f16 split scales each operand by a power of two from its
    max |x| into [2^14, 2^15)): tiny / huge / near-denormal / all-zero operands, a row block 2^-20
    below the rest and a zero row, on every complex64 K-outer kernel, against complex128 —
    2e-5 of max|C| (or exactly zero)."""
    import tneq_qc_amd.ops as ops
    rng = np.random.default_rng(5)
    M, N, K = 256, 128, 512
    a = (_rand(rng, (1, K, M), "complex128") * sa)
    b = (_rand(rng, (1, K, N), "complex128") * sb)
    a[:, :, :64] *= 2.0 ** -20
    b[:, 7, :] = 0
    a, b = a.astype("complex64"), b.astype("complex64")
    cd = _to(T, dev, np.zeros((1, M, N), "complex64"))
    ops.gemm(_to(T, dev, a), _to(T, dev, b), True, False, out=cd)
    ref = np.matmul(np.swapaxes(a.astype("complex128"), 1, 2), b.astype("complex128"))
    got = cd.cpu().numpy()
    assert np.isfinite(got).all()
    if sb == 0.0:
        assert np.all(got == 0)
        return
    err = np.abs(got - ref).max() / np.abs(ref).max()
    assert err < TOL["complex64"], (sa, sb, err)
    # the 2^-20 row block keeps its own relative accuracy (no flush of the small values) where
    # its products are f32-normal
    if np.abs(ref[:, :64]).max() > 1e-30:
        blk = np.abs(got[:, :64] - ref[:, :64]).max() / np.abs(ref[:, :64]).max()
        assert blk < 1e-4, (sa, sb, blk)


@pytest.mark.parametrize("dt", ["float64", "complex128"])
@pytest.mark.parametrize("M,N,K,B,beta", [(128, 128, 32, 1, 0.0), (256, 256, 48, 3, 0.0),
                                           (512, 256, 4096, 1, 1.0), (1024, 1024, 8192, 1, 0.0),
                                           (256, 256, 2048, 2, 0.5), (384, 384, 1024, 1, 0.0)])
def test_gemm_f64_kouter_fast_path(T, dev, dt, M, N, K, B, beta):
    """float64 / complex128 with A stored K x M and B stored K x N: the LDS-DMA v_mfma_f64 kernel
    (3-stage ring, split-K slabs, Gauss 3M for complex128) — tile-grid shapes, batched, beta."""
    import tneq_qc_amd.ops as ops
    rng = np.random.default_rng(11)
    a = _rand(rng, (B, K, M), dt)
    b = _rand(rng, (B, K, N), dt)
    c0 = _rand(rng, (B, M, N), dt)
    cd = _to(T, dev, c0)
    ops.gemm(_to(T, dev, a), _to(T, dev, b), True, False, out=cd, beta=beta)
    ref = np.matmul(np.swapaxes(a, 1, 2), b) + beta * c0
    err = np.abs(cd.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err < TOL[dt], (dt, M, N, K, B, err)


def test_gemm_c64_bench_shape(T, dev, c64_kernel):
    """The exact boundary GEMM of the C4g path (C4 before deferred tails) (M = N = 1024, K = 65536 per slice, complex64, both
    operands K-outer; the library splits K 4 ways over the workspace, as in the plan) on random
    operands, against complex128 on a sample of 64 rows (all columns): 2e-5 of max|C|."""
    import tneq_qc_amd._lib as _lib
    import tneq_qc_amd.ops as ops
    M = N = 1024
    K = 65536
    wsb = _lib.lib().tq_gemm_workspace_size(_lib.TQ_C64, M, N, K, 1)
    # componentwise too (the split terms are exact; the products keep 2^-16 relative terms): every
    # entry of the sampled rows above 1e-2 max|C| within 2e-3 relative
    assert wsb >= 4 * M * N * 8   # room for split-K 4, as in the bench
    rng = np.random.default_rng(8)
    a = _rand(rng, (1, K, M), "complex64")
    b = _rand(rng, (1, K, N), "complex64")
    c = ops.gemm(_to(T, dev, a), _to(T, dev, b), True, False).cpu().numpy()[0]
    rows = rng.choice(M, size=64, replace=False)
    ref = a[0][:, rows].T.astype("complex128") @ b[0].astype("complex128")
    err = np.abs(c[rows] - ref).max() / np.abs(ref).max()
    assert err < TOL["complex64"], err
    big = np.abs(ref) >= 1e-2 * np.abs(ref).max()
    comp = (np.abs(c[rows] - ref)[big] / np.abs(ref[big])).max()
    assert comp < TOL["complex64"] * 100, comp


def test_gemm_c64_batched_entry_scales(T, dev, c64_kernel):
    """A batched complex64 K-outer GEMM whose batch entries (the slice lanes of one plan launch)
    differ in magnitude by up to 2^50: every entry keeps its own complex64 accuracy against
    complex128 (the f16 split scales each batch entry by its own operand max; one max per launch
    would flush the small entries' terms)."""
    import tneq_qc_amd.ops as ops
    rng = np.random.default_rng(12)
    M, N, K, B = 256, 256, 2048, 4
    a = _rand(rng, (B, K, M), "complex128")
    b = _rand(rng, (B, K, N), "complex128")
    a[1] *= 2.0 ** -30
    b[1] *= 2.0 ** -20
    a[2] *= 2.0 ** 20
    b[3] *= 2.0 ** -25
    a, b = a.astype("complex64"), b.astype("complex64")
    c = ops.gemm(_to(T, dev, a), _to(T, dev, b), True, False).cpu().numpy()
    ref = np.matmul(np.swapaxes(a.astype("complex128"), 1, 2), b.astype("complex128"))
    for i in range(B):
        err = np.abs(c[i] - ref[i]).max() / np.abs(ref[i]).max()
        assert err < TOL["complex64"], (i, err)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,N,K,B,beta", [(4, 4, 16384, 1, 0.0), (8, 2, 8192, 2, 0.5), (2, 8, 512, 1, 1.0),
                                           (1, 1, 100, 3, 0.0), (16, 1, 3000, 1, 0.0), (4, 4, 64, 2, 0.0),
                                           (1, 16, 70000, 1, 0.0)])
def test_gemm_skinny(T, dev, dt, M, N, K, B, beta):
    """The skinny contraction path (M * N <= 16, M and N powers of two, long K: the reverse-mode
    gradient steps of the C5 training loop) in all four transpositions, batched, with beta, K
    not a multiple of the block range, against the exact product."""
    import tneq_qc_amd.ops as ops
    rng = np.random.default_rng(K + M)
    for ta, tb in itertools.product((False, True), (False, True)):
        a = _rand(rng, (B, K, M) if ta else (B, M, K), dt)
        b = _rand(rng, (B, N, K) if tb else (B, K, N), dt)
        c0 = _rand(rng, (B, M, N), dt)
        cd = _to(T, dev, c0)
        ops.gemm(_to(T, dev, a), _to(T, dev, b), ta, tb, out=cd, beta=beta)
        hi = "complex128" if dt.startswith("complex") else "float64"
        aa = np.swapaxes(a, 1, 2) if ta else a
        bb = np.swapaxes(b, 1, 2) if tb else b
        ref = np.matmul(aa.astype(hi), bb.astype(hi)) + beta * c0.astype(hi)
        err = np.abs(cd.cpu().numpy() - ref).max() / np.abs(ref).max()
        assert err < TOL[dt], (ta, tb, err)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("nm,nn,nk", [(2, 2, 12), (3, 1, 10), (0, 4, 9), (1, 0, 14), (4, 0, 8)])
def test_skinny_strided_step(T, dev, dt, nm, nn, nk):
    """A pairwise step with a tiny result (2^(nm+nn) <= 16 elements) whose operands would need
    permutes: the plan reads both in place through per-bit strides (SKINNY op), modes in shuffled
    orders on both sides, against numpy's einsum in the exact dtype."""
    from tneq_qc_amd.einsum import get_symbol
    from tneq_qc_amd.expression import HipContractExpression
    rng = np.random.default_rng(nm * 100 + nn * 10 + nk)
    kk = list(range(nk))
    mm = list(range(nk, nk + nm))
    nnm = list(range(nk + nm, nk + nm + nn))
    a_modes = list(rng.permutation(kk + mm))
    b_modes = list(rng.permutation(kk + nnm))
    out = list(rng.permutation(mm + nnm)) if (nm + nn) else []
    sym = lambda ms: "".join(get_symbol(int(m)) for m in ms)
    eq = f"{sym(a_modes)},{sym(b_modes)}->{sym(out)}"
    a = _rand(rng, (2,) * len(a_modes), dt)
    b = _rand(rng, (2,) * len(b_modes), dt)
    e = HipContractExpression(eq, a.shape, b.shape, optimize=[(0, 1)])
    desc = e.plan(T.from_numpy(a).dtype).describe()
    assert "SKINNY" in desc, desc
    got = e(_to(T, dev, a), _to(T, dev, b)).cpu().numpy()
    hi = "complex128" if dt.startswith("complex") else "float64"
    ref = np.einsum(eq, a.astype(hi), b.astype(hi))
    err = np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30)
    assert err < TOL[dt], (eq, err)
