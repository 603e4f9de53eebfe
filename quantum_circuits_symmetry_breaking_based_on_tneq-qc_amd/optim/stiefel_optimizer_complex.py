"""SGDG on the MI355X: drop-in for tneq_qc.optim.stiefel_optimizer_complex.SGDG
(tneq_qc/optim/stiefel_optimizer_complex.py:23-176), the optimizer the symmetry-breaking loop
steps after every backward pass (symmetry_breaking_quantum.py:156,203,216-230).

Same constructor, same param_groups / state layout (state[p]['momentum_buffer']), same branch
rule and the same host-side random draw: for every parameter with a gradient, viewed as
rows x cols = prod(size[:ndim//2]) x prod(size[ndim//2:]), the Stiefel (Cayley) branch runs when
stiefel=True and rows <= cols, drawing random.randint(1, 101) from Python's global `random`
exactly where the reference does (a 1 triggers qr_retraction of the row-normalised
parameter); every other parameter takes the SGD branch (weight decay / momentum / dampening /
nesterov, the gradient updated in place by the weight decay as d_p.add_ does).
The arithmetic of a whole group is ONE native launch (tq_sgdg_step: one workgroup per
parameter, every matrix LDS-resident up to 32 columns and on a global scratch above -- 1-D
parameters are 1 x len, cores of bond dimension >= 3 have cols >= 9 --, the Cayley solve by
Gauss-Jordan) instead of ~20 small torch launches per parameter.  Parameters must live on the
HIP device; there is no CPU path.  Every parameter of every group is checked (device, dtype,
layout, Stiefel shape limit) before any random draw, state change or launch, so an unsupported
parameter raises with the optimizer and the parameters untouched.
"""
from __future__ import annotations

import ctypes
import random

import torch
from torch.optim.optimizer import Optimizer, required

from .. import _lib

_DT = {torch.float32: _lib.TQ_F32, torch.float64: _lib.TQ_F64,
       torch.complex64: _lib.TQ_C64, torch.complex128: _lib.TQ_C128}
MAX_STIEFEL_COLS = 2048   # TQ_SGDG_MAX_COLS (include/tneqhip.h)


def _view_dims(size):
    nd = len(size)
    mid = nd // 2
    rows = 1
    for s in size[:mid]:
        rows *= int(s)
    cols = 1
    for s in size[mid:]:
        cols *= int(s)
    return rows, cols


class SGDG(Optimizer):
    def __init__(self, params, lr=required, momentum=0, dampening=0, weight_decay=0,
                 nesterov=False, stiefel=False, omega=0, grad_clip=None, rng=None):
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, stiefel=stiefel, omega=0, grad_clip=grad_clip)
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, defaults)
        # source of the retraction draws: Python's global `random` (the reference's), or a
        # random.Random of the caller's (e.g. one stream per concurrently trained candidate)
        self._rng = rng

    def __setstate__(self, state):
        super().__setstate__(state)
        for group in self.param_groups:
            group.setdefault("nesterov", False)

    def _launch_group(self, group, items_by_batch, flags_by_batch):
        L = _lib.lib()
        for (dtype, dev), arrs in items_by_batch.items():
            n, vp, vg, vb, ir, ic = arrs
            flags = (ctypes.c_int32 * n)(*flags_by_batch[(dtype, dev)])
            stream = torch.cuda.current_stream(dev).cuda_stream
            with torch.cuda.device(dev):
                _lib.check(L.tq_sgdg_step(
                    _DT[dtype], n, vp, vg, vb, ir, ic, flags, float(group["lr"]),
                    float(group["momentum"]), float(group["dampening"]), float(group["weight_decay"]),
                    int(bool(group["nesterov"])), ctypes.c_void_p(stream)), "sgdg_step")

    def _cache_key(self, group):
        key = []
        for p in group["params"]:
            g = p.grad
            buf = self.state[p].get("momentum_buffer") if p in self.state else None
            key.append((id(p), p.data_ptr(), g.data_ptr() if g is not None else 0,
                        buf.data_ptr() if buf is not None else 0))
        return (tuple(key), group["stiefel"], group["momentum"])

    def _fast_flags(self, group, masks):
        """Per-step flags of a cached group: the random draws in parameter order, exactly where
        the reference draws (stiefel_optimizer_complex.py:111-113)."""
        flags_by_batch = {}
        rng = self._rng if getattr(self, "_rng", None) is not None else random
        mom = _lib.TQ_SGDG_BUF_INIT if group["momentum"] != 0 else 0
        for bk, stiefel_mask in masks.items():
            fl = []
            for st in stiefel_mask:
                if st:
                    f = _lib.TQ_SGDG_STIEFEL | _lib.TQ_SGDG_BUF_INIT
                    if rng.randint(1, 101) == 1:
                        f |= _lib.TQ_SGDG_RETRACT
                    fl.append(f)
                else:
                    fl.append(mom)
            flags_by_batch[bk] = fl
        return flags_by_batch

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        # Steady state (a training loop: the same parameters, gradients and momentum buffers
        # every step): a group's checks, per-parameter views and launch pointer arrays are cached,
        # keyed by every parameter's, gradient's and buffer's identity / address; only the random
        # draws and the flags are per step.  When every group hits, no check can fail.
        cache = getattr(self, "_sgdg_cache", {})
        hits = [cache.get(gi) is not None and cache[gi][0] == self._cache_key(g)
                for gi, g in enumerate(self.param_groups)]
        if all(hits):
            for gi, group in enumerate(self.param_groups):
                self._launch_group(group, cache[gi][1], self._fast_flags(group, cache[gi][2]))
            return loss
        L = _lib.lib()
        # every parameter is checked before anything is drawn, created or launched
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.device.type != "cuda":
                    raise ValueError("SGDG (HIP) needs parameters on the HIP device")
                if p.dtype not in _DT:
                    raise ValueError(f"SGDG (HIP): unsupported dtype {p.dtype}")
                if not p.is_contiguous() or not p.grad.is_contiguous():
                    raise ValueError("SGDG (HIP) needs contiguous parameters and gradients")
                rows, cols = _view_dims(p.size())
                if group["stiefel"] and rows <= cols and cols > MAX_STIEFEL_COLS:
                    raise ValueError(f"SGDG (HIP): Stiefel parameter {tuple(p.size())} has {cols} columns "
                                     f"(at most {MAX_STIEFEL_COLS})")
        rng = self._rng if getattr(self, "_rng", None) is not None else random
        for group in self.param_groups:
            momentum, stiefel = group["momentum"], group["stiefel"]
            batches = {}   # (dtype, device) -> list of descriptors, in parameter order
            for p in group["params"]:
                if p.grad is None:
                    continue
                rows, cols = _view_dims(p.size())
                st = self.state[p]
                flags = 0
                if stiefel and rows <= cols:
                    flags |= _lib.TQ_SGDG_STIEFEL
                    if rng.randint(1, 101) == 1:          # stiefel_optimizer_complex.py:111-113
                        flags |= _lib.TQ_SGDG_RETRACT
                    if "momentum_buffer" not in st:
                        st["momentum_buffer"] = torch.zeros((cols, rows), dtype=p.dtype, device=p.device)
                    flags |= _lib.TQ_SGDG_BUF_INIT
                elif momentum != 0:
                    if "momentum_buffer" not in st:
                        st["momentum_buffer"] = torch.empty_like(p)   # kernel writes d_p.clone()
                    else:
                        flags |= _lib.TQ_SGDG_BUF_INIT
                buf = st.get("momentum_buffer")
                batches.setdefault((p.dtype, p.device), []).append((p, buf, rows, cols, flags))
            arrays, flags_by_batch, masks = {}, {}, {}
            for (dtype, dev), items in batches.items():
                n = len(items)
                VP = ctypes.c_void_p * n
                I32 = ctypes.c_int32 * n
                arrays[(dtype, dev)] = (
                    n, VP(*[it[0].data_ptr() for it in items]), VP(*[it[0].grad.data_ptr() for it in items]),
                    VP(*[(it[1].data_ptr() if it[1] is not None else 0) for it in items]),
                    I32(*[it[2] for it in items]), I32(*[it[3] for it in items]))
                flags_by_batch[(dtype, dev)] = [it[4] for it in items]
                masks[(dtype, dev)] = [bool(it[4] & _lib.TQ_SGDG_STIEFEL) for it in items]
            self._launch_group(group, arrays, flags_by_batch)
            # cached for the steady state only when the cached draw order (batch-major) is
            # parameter order: one batch (a single dtype / device)
            gi = next(k for k, g in enumerate(self.param_groups) if g is group)
            if not hasattr(self, "_sgdg_cache"):
                self._sgdg_cache = {}
            if len(batches) == 1:
                self._sgdg_cache[gi] = (self._cache_key(group), arrays, masks)
            else:
                self._sgdg_cache.pop(gi, None)
        return loss
