"""HipContractExpression: the drop-in for ``opt_einsum.contract_expression(eq, *shapes)``.

The reference builds one einsum equation per network and evaluates it with
``opt_einsum.contract_expression(eq, *shapes, optimize=...)`` followed by ``expr(*tensors)``
(tneq_qc/contractor/einsum_strategy.py:622-643; symmetry_breaking_quantum.py:142-144, 213-221;
executed through ComputeBackend.execute_expression, backend_interface.py:102-114).  Here the same
call shape returns an object whose ``__call__`` runs the whole pairwise tree on the MI355X through
one native plan (libtneqhip ``tq_plan_*``): intermediates live in a preallocated HBM arena, every
pairwise step is lowered to APPLY / permute+MFMA-GEMM kernels on the current torch stream.
Index slicing is a first-class option: ``slices=[symbols]`` removes those
contracted symbols from the inputs and sums the sub-contractions.
"""
from __future__ import annotations

import ctypes
import threading
from typing import Dict, List, Optional, Sequence, Tuple, Union

import torch

from . import _lib
from ._lib import check, i32, i64
from .einsum import (Network, greedy_path, linear_path, parse_equation, path_info,
                     validate_path)
from .ops import dtype_code

PathSpec = Union[str, Sequence[Tuple[int, int]]]


class NativePlan:
    """Owner of one ``tq_plan`` (compiled for a dtype + input strides; arena allocated lazily)."""

    def __init__(self, net: Network, path: Sequence[Tuple[int, int]], dtype: torch.dtype,
                 strides: Optional[Sequence[Sequence[int]]], sliced: Sequence[int]):
        L = _lib.lib()
        ranks = [len(t) for t in net.terms]
        modes = [m for t in net.terms for m in t]
        exts = [net.extents[m] for t in net.terms for m in t]
        st = None
        if strides is not None:
            st = i64([s for ss in strides for s in ss])
        flat_path = [x for p in path for x in p]
        h = ctypes.c_void_p()
        rc = L.tq_plan_create(ctypes.byref(h), dtype_code(dtype), len(net.terms), i32(ranks),
                              i32(modes), i64(exts), st, len(net.out), i32(net.out), len(path),
                              i32(flat_path), len(sliced), i32(sliced))
        check(rc, "tq_plan_create")
        self._h = h
        self.dtype = dtype
        self.n_slices = self.query("n_slices")

    def query(self, key: str) -> int:
        return int(_lib.lib().tq_plan_query(self._h, key.encode()))

    def describe(self) -> str:
        L = _lib.lib()
        n = L.tq_plan_describe(self._h, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        L.tq_plan_describe(self._h, buf, n + 1)
        return buf.value.decode()

    def execute(self, ptrs: Sequence[int], out_ptr: int, stream: int, begin: int = 0,
                end: Optional[int] = None, step: int = 1, accumulate: bool = False) -> None:
        end = self.n_slices if end is None else end
        arr = (ctypes.c_void_p * max(1, len(ptrs)))(*[ctypes.c_void_p(p) for p in ptrs])
        rc = _lib.lib().tq_plan_execute(self._h, arr, ctypes.c_void_p(out_ptr), begin, end, step,
                                        int(accumulate), ctypes.c_void_p(stream))
        check(rc, "tq_plan_execute")

    def profile(self, kinds=-1) -> None:
        """Reset the records and time (HIP events on the execution stream) the op kinds in
        `kinds` (one _lib.TQ_OP_* or an iterable of them; -1 = all; None / [] = off)."""
        if kinds is None:
            mask = 0
        elif isinstance(kinds, int):
            mask = -1 if kinds == -1 else (1 << kinds)
        else:
            mask = 0
            for k in kinds:
                mask |= 1 << int(k)
        check(_lib.lib().tq_plan_profile(self._h, int(mask)), "tq_plan_profile")

    def profile_read(self, op_kind: int = -1) -> dict:
        """Summed event time / launches / algorithmic flops and bytes of one op kind
        (_lib.TQ_OP_GEMM, TQ_OP_APPLY, TQ_OP_PERMUTE; -1 = all) since the last reset."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        fl, by = ctypes.c_double(), ctypes.c_double()
        check(_lib.lib().tq_plan_profile_read(self._h, op_kind, ctypes.byref(ms), ctypes.byref(n),
                                              ctypes.byref(fl), ctypes.byref(by)), "tq_plan_profile_read")
        return {"ms": ms.value, "launches": n.value, "flops": fl.value, "bytes": by.value}

    def __del__(self):
        try:
            h = getattr(self, "_h", None)
            if h is not None and _lib._lib is not None:
                _lib._lib.tq_plan_destroy(h)
                self._h = None
        except Exception:  # interpreter shutdown: modules may already be gone
            pass


class HipContractExpression:
    """Callable contraction of a fixed einsum equation over fixed shapes on the HIP engine.

    ``optimize``: 'greedy' / 'auto' (opt_einsum's greedy rule), 'linear' (sweep with `order`
    hint), or an explicit SSA path [(i, j), ...].  ``slices``: symbols (or mode ids) to slice.
    """

    def __init__(self, eq: str, *shapes, optimize: PathSpec = "greedy",
                 order: Optional[Sequence[int]] = None, slices: Sequence = ()):
        self.eq = eq
        self.shapes = [tuple(int(x) for x in s) for s in shapes]
        self.net = parse_equation(eq, self.shapes)
        n = len(self.net.terms)
        if isinstance(optimize, str):
            if optimize in ("greedy", "auto", "optimal", "dp", "branch-2", "random-greedy"):
                self.path = greedy_path(self.net) if n > 1 else []
            elif optimize == "linear":
                self.path = linear_path(self.net, order)[0] if n > 1 else []
            else:
                raise ValueError(f"unknown optimize={optimize!r}")
        else:
            self.path = [tuple(int(x) for x in p) for p in optimize]
        validate_path(n, self.path)
        sym2id = {s: i for i, s in enumerate(self.net.symbols)}
        self.sliced = [sym2id[s] if isinstance(s, str) else int(s) for s in slices]
        for m in self.sliced:
            if m in self.net.out:
                raise ValueError("cannot slice an output symbol")
        self.n_slices = 1
        for m in self.sliced:
            self.n_slices *= self.net.extents[m]
        self._plans: Dict[tuple, NativePlan] = {}
        self._lock = threading.Lock()

    # -- introspection ---------------------------------------------------------------------
    @property
    def out_shape(self) -> Tuple[int, ...]:
        return tuple(self.net.extents[m] for m in self.net.out)

    def info(self):
        return path_info(self.net, self.path, self.sliced)

    def plan(self, dtype: torch.dtype, strides=None, device: Optional[int] = None) -> NativePlan:
        """The native plan for (dtype, input strides, device).  A plan's arena, tables and graphs
        live on the device that was current at its first execute; the library refuses to run it
        with another device current, so plans are keyed by device.  One plan serves one stream
        at a time (its arena is shared by its launches)."""
        if device is None:
            device = torch.cuda.current_device() if torch.cuda.is_available() else -1
        key = (dtype, None if strides is None else tuple(tuple(s) for s in strides), int(device))
        p = self._plans.get(key)
        if p is None:
            with self._lock:
                p = self._plans.get(key)
                if p is None:
                    p = NativePlan(self.net, self.path, dtype, strides, self.sliced)
                    self._plans[key] = p
        return p

    # -- execution ---------------------------------------------------------------------------
    def __call__(self, *tensors, out: Optional[torch.Tensor] = None, slice_range=None,
                 accumulate: bool = False, backend=None) -> torch.Tensor:
        if (torch.is_grad_enabled() and out is None and slice_range is None
                and any(isinstance(t, torch.Tensor) and t.requires_grad for t in tensors)):
            return _HipContractFn.apply(self, *tensors)
        return self._forward(*tensors, out=out, slice_range=slice_range, accumulate=accumulate)

    def grad_expression(self, i: int) -> Tuple["HipContractExpression", List[int]]:
        """Expression for d(out)/d(operand i) contracted with grad_out:
        operands = the other inputs (conjugated by the caller) + grad_out -> operand i's modes.
        Modes only present in operand i are broadcast afterwards (returned as positions)."""
        key = ("grad", i)
        hit = self._plans.get(key)
        if hit is not None:
            return hit
        sym = self.net.symbols
        others = [j for j in range(len(self.net.terms)) if j != i]
        present = set(self.net.out)
        for j in others:
            present |= set(self.net.terms[j])
        term_i = self.net.terms[i]
        kept = [m for m in term_i if m in present]
        bcast = [k for k, m in enumerate(term_i) if m not in present]
        eq = ",".join("".join(sym[m] for m in self.net.terms[j]) for j in others)
        eq += ("," if others else "") + "".join(sym[m] for m in self.net.out)
        eq += "->" + "".join(sym[m] for m in kept)
        shapes = [self.shapes[j] for j in others] + [self.out_shape]
        g = HipContractExpression(eq, *shapes, optimize="greedy")
        self._plans[key] = (g, bcast)
        return g, bcast

    def _forward(self, *tensors, out: Optional[torch.Tensor] = None, slice_range=None,
                 accumulate: bool = False) -> torch.Tensor:
        if len(tensors) != len(self.net.terms):
            raise ValueError(f"expression takes {len(self.net.terms)} operands, got {len(tensors)}")
        ts = [t if isinstance(t, torch.Tensor) else torch.as_tensor(t) for t in tensors]
        for t, s in zip(ts, self.shapes):
            if tuple(t.shape) != s:
                raise ValueError(f"operand shape {tuple(t.shape)} does not match expression shape {s}")
        dev = next((t.device for t in ts if t.device.type == "cuda"), None)
        if dev is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        dt = ts[0].dtype
        for t in ts[1:]:
            dt = torch.promote_types(dt, t.dtype)
        dtype_code(dt)
        # torch's lazy conj/neg bits are not visible through data_ptr(): materialise them
        ts = [t.to(device=dev, dtype=dt).resolve_conj().resolve_neg() for t in ts]
        # views with odd strides are fine (the plan reads through strides); negative/overlap not
        ts = [t if all(s >= 0 for s in t.stride()) else t.contiguous() for t in ts]
        strides = [t.stride() for t in ts]
        contiguous = all(t.is_contiguous() for t in ts)
        plan = self.plan(dt, None if contiguous else strides, dev.index)
        if out is None:
            out = torch.empty(self.out_shape, dtype=dt, device=dev)
            accumulate = False
        elif (tuple(out.shape) != self.out_shape or out.dtype != dt or not out.is_contiguous()
              or out.device != dev):
            raise ValueError("out tensor has the wrong shape/dtype/device or is not contiguous")
        begin, end, step = (0, plan.n_slices, 1) if slice_range is None else slice_range
        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev).cuda_stream
            plan.execute([t.data_ptr() for t in ts], out.data_ptr(), stream, begin, end, step, accumulate)
        return out


class _HipContractFn(torch.autograd.Function):
    """Autograd for a HIP expression: d/d(operand i) = contraction of grad_out with the
    conjugated other operands (torch's convention for complex einsum), each on the HIP engine."""

    @staticmethod
    def forward(ctx, expr, *tensors):
        ctx.expr = expr
        ctx.save_for_backward(*[t if isinstance(t, torch.Tensor) else torch.as_tensor(t) for t in tensors])
        with torch.no_grad():
            return expr._forward(*[t.detach() if isinstance(t, torch.Tensor) else t for t in tensors])

    @staticmethod
    def backward(ctx, grad_out):
        expr = ctx.expr
        ts = ctx.saved_tensors
        grads = [None]
        for i, t in enumerate(ts):
            if not ctx.needs_input_grad[i + 1]:
                grads.append(None)
                continue
            g_expr, bcast = expr.grad_expression(i)
            others = [torch.conj_physical(ts[j]) if ts[j].is_complex() else ts[j]
                      for j in range(len(ts)) if j != i]
            g = g_expr._forward(*others, grad_out.to(dtype=torch.promote_types(grad_out.dtype, t.dtype)))
            for k in bcast:
                g = g.unsqueeze(k)
            g = g.expand(t.shape)
            grads.append(g.to(device=t.device, dtype=t.dtype))
        return tuple(grads)


def contract_expression(eq: str, *shapes, optimize: PathSpec = "greedy", **kw) -> HipContractExpression:
    """Same call shape as ``opt_einsum.contract_expression`` (einsum_strategy.py:639-643)."""
    return HipContractExpression(eq, *shapes, optimize=optimize, **kw)


def contract(eq: str, *tensors, optimize: PathSpec = "greedy", **kw) -> torch.Tensor:
    """One-shot einsum on the HIP engine (``opt_einsum.contract`` / ``torch.einsum`` drop-in)."""
    expr = HipContractExpression(eq, *[tuple(t.shape) for t in tensors], optimize=optimize, **kw)
    return expr(*tensors)
