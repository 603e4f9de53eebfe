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
                 nesterov=False, stiefel=False, omega=0, grad_clip=None):
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, stiefel=stiefel, omega=0, grad_clip=grad_clip)
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, defaults)

    def __setstate__(self, state):
        super().__setstate__(state)
        for group in self.param_groups:
            group.setdefault("nesterov", False)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
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
                    if random.randint(1, 101) == 1:       # stiefel_optimizer_complex.py:111-113
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
            for (dtype, dev), items in batches.items():
                n = len(items)
                VP = ctypes.c_void_p * n
                I32 = ctypes.c_int32 * n
                stream = torch.cuda.current_stream(dev).cuda_stream
                with torch.cuda.device(dev):
                    _lib.check(L.tq_sgdg_step(
                        _DT[dtype], n, VP(*[it[0].data_ptr() for it in items]),
                        VP(*[it[0].grad.data_ptr() for it in items]),
                        VP(*[(it[1].data_ptr() if it[1] is not None else 0) for it in items]),
                        I32(*[it[2] for it in items]), I32(*[it[3] for it in items]),
                        I32(*[it[4] for it in items]), float(group["lr"]), float(momentum),
                        float(group["dampening"]), float(group["weight_decay"]),
                        int(bool(group["nesterov"])), ctypes.c_void_p(stream)), "sgdg_step")
        return loss
