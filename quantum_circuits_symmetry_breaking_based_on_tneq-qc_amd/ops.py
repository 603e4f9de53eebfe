"""torch-tensor entry points over the C ABI (device memory and streams come from torch).

These are the device primitives the backend and the contraction plans are built from:
``permute`` (reference: BackendPyTorch.permute, tneq_qc/backends/backend_pytorch.py:619-621),
``gemm`` (the GEMM under every tensordot), ``contract_pair`` (one pairwise einsum,
BackendPyTorch.einsum with two operands, backend_pytorch.py:623-625), and the measurement-data
kernels of EngineSiamese: ``hermite_features`` (generate_data, engine_siamese.py:133-254) and
``inverse_cdf_sample`` (the CDF block of sample, engine_siamese.py:854-905).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check, i32, i64

_DT = {
    torch.float32: _lib.TQ_F32,
    torch.float64: _lib.TQ_F64,
    torch.complex64: _lib.TQ_C64,
    torch.complex128: _lib.TQ_C128,
}


def dtype_code(dtype: torch.dtype) -> int:
    try:
        return _DT[dtype]
    except KeyError:
        raise ValueError(f"unsupported dtype {dtype}; supported: float32, float64, complex64, complex128")


def _stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _require_device(*ts: torch.Tensor) -> torch.device:
    dev = ts[0].device
    if dev.type != "cuda":
        raise ValueError(f"tensors must be on a HIP device (got {dev}); use BackendHIP.convert_to_tensor")
    for t in ts[1:]:
        if t.device != dev:
            raise ValueError("all operands must live on the same device")
        if t.dtype != ts[0].dtype:
            raise ValueError("all operands must have the same dtype")
    return dev


def permute(x: torch.Tensor, dims: Sequence[int]) -> torch.Tensor:
    """Materialised ``x.permute(dims).contiguous()`` through the LDS-tiled HIP kernel."""
    dev = _require_device(x)
    dims = [int(d) % max(1, x.ndim) for d in dims]
    if sorted(dims) != list(range(x.ndim)):
        raise ValueError(f"invalid permutation {dims} for rank {x.ndim}")
    shape = [x.shape[d] for d in dims]
    strides = [x.stride(d) for d in dims]
    out = torch.empty(shape, dtype=x.dtype, device=dev)
    if out.numel() == 0:
        return out
    rc = _lib.lib().tq_permute(dtype_code(x.dtype), len(shape), i64(shape), i64(strides),
                               ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                               0.0, ctypes.c_void_p(_stream_ptr(dev)))
    check(rc, "tq_permute")
    return out


def gemm(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False, trans_b: bool = False,
         out: torch.Tensor | None = None, beta: float = 0.0) -> torch.Tensor:
    """Batched ``C = op(A) @ op(B) (+ beta*C)`` on MFMA; a, b are 2-D or 3-D (batch first), contiguous."""
    dev = _require_device(a, b)
    a3 = a if a.ndim == 3 else a.unsqueeze(0)
    b3 = b if b.ndim == 3 else b.unsqueeze(0)
    if not (a3.is_contiguous() and b3.is_contiguous()):
        raise ValueError("gemm operands must be contiguous")
    batch = a3.shape[0]
    if b3.shape[0] != batch:
        raise ValueError("batch mismatch")
    M, K = (a3.shape[2], a3.shape[1]) if trans_a else (a3.shape[1], a3.shape[2])
    Kb, N = (b3.shape[2], b3.shape[1]) if trans_b else (b3.shape[1], b3.shape[2])
    if K != Kb:
        raise ValueError(f"inner dimension mismatch {K} vs {Kb}")
    if out is None:
        out = torch.empty((batch, M, N), dtype=a.dtype, device=dev)
        beta = 0.0
    out3 = out if out.ndim == 3 else out.unsqueeze(0)
    code = dtype_code(a.dtype)
    L = _lib.lib()
    wsb = L.tq_gemm_workspace_size(code, M, N, K, batch)
    ws = torch.empty(max(1, wsb), dtype=torch.uint8, device=dev) if wsb else None
    rc = L.tq_gemm_batched(code, int(trans_a), int(trans_b), M, N, K, batch,
                           ctypes.c_void_p(a3.data_ptr()), a3.shape[2], a3.shape[1] * a3.shape[2],
                           ctypes.c_void_p(b3.data_ptr()), b3.shape[2], b3.shape[1] * b3.shape[2],
                           float(beta), ctypes.c_void_p(out3.data_ptr()), N, M * N,
                           ctypes.c_void_p(ws.data_ptr() if ws is not None else 0), wsb,
                           ctypes.c_void_p(_stream_ptr(dev)))
    check(rc, "tq_gemm_batched")
    if a.ndim == 2 and b.ndim == 2 and out.ndim == 3:
        return out3[0]
    return out


def contract_pair(modes_a: Sequence[int], a: torch.Tensor, modes_b: Sequence[int], b: torch.Tensor,
                  modes_c: Sequence[int]) -> torch.Tensor:
    """einsum("A,B->C") with integer mode labels, on the HIP engine."""
    dev = _require_device(a, b)
    a = a.contiguous()
    b = b.contiguous()
    ext = {}
    for m, e in list(zip(modes_a, a.shape)) + list(zip(modes_b, b.shape)):
        if ext.setdefault(int(m), int(e)) != int(e):
            raise ValueError(f"mode {m} has inconsistent extents")
    try:
        shape_c = [ext[int(m)] for m in modes_c]
    except KeyError as e:
        raise ValueError(f"output mode {e} not present in inputs")
    out = torch.empty(shape_c, dtype=a.dtype, device=dev)
    code = dtype_code(a.dtype)
    L = _lib.lib()
    args = (code, len(modes_a), i64(a.shape), i32(modes_a), len(modes_b), i64(b.shape), i32(modes_b),
            len(modes_c), i32(modes_c))
    wsb = L.tq_contract_pair_workspace(*args)
    if wsb == 0:
        raise ValueError(f"contract_pair: {_lib.last_error()}")
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    rc = L.tq_contract_pair(code, len(modes_a), i64(a.shape), i32(modes_a), ctypes.c_void_p(a.data_ptr()),
                            len(modes_b), i64(b.shape), i32(modes_b), ctypes.c_void_p(b.data_ptr()),
                            len(modes_c), i32(modes_c), ctypes.c_void_p(out.data_ptr()),
                            ctypes.c_void_p(ws.data_ptr()), wsb, ctypes.c_void_p(_stream_ptr(dev)))
    check(rc, "tq_contract_pair")
    return out


def axpy(x: torch.Tensor, y: torch.Tensor, beta: float = 1.0) -> torch.Tensor:
    """y = x + beta*y in place (partial-amplitude accumulation)."""
    dev = _require_device(x, y)
    if x.numel() != y.numel() or not (x.is_contiguous() and y.is_contiguous()):
        raise ValueError("axpy needs equal-size contiguous tensors")
    rc = _lib.lib().tq_axpy(dtype_code(x.dtype), x.numel(), ctypes.c_void_p(x.data_ptr()),
                            ctypes.c_void_p(y.data_ptr()), float(beta), ctypes.c_void_p(_stream_ptr(dev)))
    check(rc, "tq_axpy")
    return y


def hermite_features(x: torch.Tensor, K: int, weights, dtype: torch.dtype, want_phi: bool = True):
    """Hermite measurement data of every entry of ``x`` (any shape; the real part is used):
    ``phi[..., k] = (w_k * sqrt(exp(-x^2/2))) * He_k(x)`` and ``mx[..., k, l] = conj(phi_k) phi_l``
    in ``dtype``; complex dtypes compute in float64, real dtypes in their own precision
    (engine_siamese.py:133-254).  ``weights``: host array of at least K float64 w_k.
    Returns (phi or None, mx)."""
    dev = _require_device(x)
    K = int(K)
    if not 1 <= K <= _lib.TQ_HERMITE_MAX_K:
        raise ValueError(f"K must be in [1, {_lib.TQ_HERMITE_MAX_K}], got {K}")
    w = np.ascontiguousarray(np.asarray(weights, dtype=np.float64).reshape(-1)[:K])
    if w.shape[0] < K:
        raise ValueError(f"need {K} Hermite weights, got {w.shape[0]}")
    xd = (x.real if x.is_complex() else x).to(torch.float64).contiguous()
    phi = torch.empty(tuple(x.shape) + (K,), dtype=dtype, device=dev) if want_phi else None
    mx = torch.empty(tuple(x.shape) + (K, K), dtype=dtype, device=dev)
    rc = _lib.lib().tq_hermite_features(dtype_code(dtype), xd.numel(), K, ctypes.c_void_p(xd.data_ptr()),
                                        w.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                        ctypes.c_void_p(phi.data_ptr() if phi is not None else None),
                                        ctypes.c_void_p(mx.data_ptr()), ctypes.c_void_p(_stream_ptr(dev)))
    check(rc, "tq_hermite_features")
    return phi, mx


def inverse_cdf_sample(density: torch.Tensor, grid: torch.Tensor, u: torch.Tensor,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One inverse-CDF draw per row of a real (S, G) density on a (G,) grid with S float32
    uniforms ``u`` (engine_siamese.py:857-905): clamp >= 0, cumsum, / (total + 1e-10),
    idx = min(#(cdf < u), G - 2), linear interpolation.  Returns (S,) in the density's dtype."""
    if density.ndim != 2 or grid.ndim != 1 or grid.shape[0] != density.shape[1]:
        raise ValueError(f"density must be (S, G) and grid (G,), got {tuple(density.shape)} and {tuple(grid.shape)}")
    if density.dtype not in (torch.float32, torch.float64):
        raise ValueError(f"density must be real float32/float64, got {density.dtype}")
    dev = _require_device(density, grid)
    S, G = density.shape
    d = density.contiguous()
    gr = grid.contiguous()
    uu = u.reshape(-1).to(device=dev, dtype=torch.float32).contiguous()
    if uu.numel() != S:
        raise ValueError(f"need {S} uniforms, got {uu.numel()}")
    if out is None:
        out = torch.empty(S, dtype=density.dtype, device=dev)
    elif out.shape != (S,) or out.dtype != density.dtype or out.device != dev:
        raise ValueError("out must be an (S,) tensor of the density's dtype on its device")
    rc = _lib.lib().tq_inverse_cdf_sample(dtype_code(density.dtype), S, G, ctypes.c_void_p(d.data_ptr()), G,
                                          ctypes.c_void_p(gr.data_ptr()), ctypes.c_void_p(uu.data_ptr()),
                                          ctypes.c_void_p(out.data_ptr()), out.stride(0),
                                          ctypes.c_void_p(_stream_ptr(dev)))
    check(rc, "tq_inverse_cdf_sample")
    return out


class _FidelityLoss(torch.autograd.Function):
    """L = 1 - |<t, o>|^2 / max(<t, t> <o, o>, 1e-12) (symmetry_breaking_quantum.py:220-229):
    one launch forward (tq_fidelity_forward), one backward (tq_fidelity_backward); the target
    gets no gradient (it is a constant of the fit)."""

    @staticmethod
    def forward(ctx, out_f, tgt_f):
        dev = _require_device(out_f, tgt_f)
        o = out_f.contiguous()
        t = tgt_f.contiguous()
        stats = torch.empty(4, dtype=torch.float64, device=dev)
        loss = torch.empty((), dtype=o.real.dtype, device=dev)
        check(_lib.lib().tq_fidelity_forward(dtype_code(o.dtype), o.numel(), ctypes.c_void_p(t.data_ptr()),
                                             ctypes.c_void_p(o.data_ptr()), ctypes.c_void_p(stats.data_ptr()),
                                             ctypes.c_void_p(loss.data_ptr()), ctypes.c_void_p(_stream_ptr(dev))),
              "tq_fidelity_forward")
        ctx.save_for_backward(o, t, stats)
        return loss

    @staticmethod
    def backward(ctx, g):
        o, t, stats = ctx.saved_tensors
        dev = o.device
        gg = g.to(dtype=o.real.dtype).contiguous()
        grad = torch.empty_like(o)
        check(_lib.lib().tq_fidelity_backward(dtype_code(o.dtype), o.numel(), ctypes.c_void_p(t.data_ptr()),
                                              ctypes.c_void_p(o.data_ptr()), ctypes.c_void_p(stats.data_ptr()),
                                              ctypes.c_void_p(gg.data_ptr()), ctypes.c_void_p(grad.data_ptr()),
                                              ctypes.c_void_p(_stream_ptr(dev))), "tq_fidelity_backward")
        return grad, None


def fidelity_loss(out: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """The symmetry-breaking fit's loss 1 - |<target, out>|^2 / max(<target, target> <out, out>,
    1e-12) over the flattened tensors (symmetry_breaking_quantum.py:220-229: vdot, abs()**2,
    clamp_min, 1 - num/den), differentiable w.r.t. ``out``; complex64 / complex128 on the HIP
    device.  Returns a 0-d real tensor."""
    if out.dtype not in (torch.complex64, torch.complex128) or target.dtype != out.dtype:
        raise ValueError(f"fidelity_loss: complex64 / complex128 operands of one dtype (got {out.dtype}, {target.dtype})")
    if out.numel() != target.numel():
        raise ValueError(f"fidelity_loss: {out.numel()} vs {target.numel()} elements")
    if target.requires_grad:
        raise ValueError("fidelity_loss: the target is a constant (no gradient)")
    return _FidelityLoss.apply(out.reshape(-1), target.reshape(-1))
