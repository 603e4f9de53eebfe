"""ORACLE (test infrastructure only): numpy restatement of SGDG.step.

Follows tneq_qc/optim/stiefel_optimizer_complex.py:77-176 line by line, with the helpers of
tneq_qc/optim/gutils.py: unit (:7-9, rows divided by their 2-norm + 1e-8), qr_retraction
(:59-78, QR of X^H with the diagonal phases of R moved into Q), matrix_norm_one (:134-138, max
column sum of |W|), and SGDG.compute_Y (:66-74, inverse(I - a/2 W) @ (I + a/2 W) @ X).
Computes in the parameter's own precision (complex64 stays complex64), as torch does.
The 1-in-101 qr_retraction draw uses Python's global `random` exactly where the reference does
(random.randint(1, 101) for every Stiefel-branch parameter, in parameter order), so seeding
`random` identically reproduces the reference's draws.
"""
from __future__ import annotations

import random
from typing import Dict, List

import numpy as np

EPS = 1e-8


def unit(v: np.ndarray, eps: float = 1e-8):                         # gutils.py:7-9
    n = np.linalg.norm(v, axis=1, keepdims=True).astype(v.real.dtype)
    return (v / (n + v.real.dtype.type(eps))).astype(v.dtype), n


def qr_retraction(x: np.ndarray) -> np.ndarray:                     # gutils.py:59-78
    t = np.conj(x).T if np.iscomplexobj(x) else x.T
    q, r = np.linalg.qr(t, mode="reduced")
    d = np.diag(r)
    if np.iscomplexobj(d):
        ph = np.where(d == 0, 0, d / np.where(d == 0, 1, np.abs(d)))
    else:
        ph = np.sign(d)
    q = q * ph[None, :]
    return (np.conj(q).T if np.iscomplexobj(x) else q.T).astype(x.dtype)


def matrix_norm_one(w: np.ndarray):                                 # gutils.py:134-138
    return np.abs(w).sum(axis=0).max()


def sgdg_step(params: List[np.ndarray], grads: List[np.ndarray], state: Dict[int, dict], lr: float,
              momentum: float = 0.0, dampening: float = 0.0, weight_decay: float = 0.0,
              nesterov: bool = False, stiefel: bool = False, rng=random):
    """One SGDG.step over `params` (updated in place, as p.data.copy_ / add_); `grads` are
    updated in place by the SGD branch's weight decay (d_p.add_).  state[i]['momentum_buffer']
    as the reference keeps it."""
    for i, (p, g) in enumerate(zip(params, grads)):
        size = p.shape
        mid = len(size) // 2
        rows = int(np.prod(size[:mid], dtype=np.int64))
        cols = int(np.prod(size[mid:], dtype=np.int64))
        dt = p.dtype
        rdt = p.real.dtype.type
        X, _ = unit(p.reshape(rows, cols))
        if stiefel and X.shape[0] <= X.shape[1]:
            if rng.randint(1, 101) == 1:                            # :111-113
                X = qr_retraction(X)
            G = g.reshape(rows, cols)
            st = state.setdefault(i, {})
            if "momentum_buffer" not in st:
                st["momentum_buffer"] = np.zeros((cols, rows), dtype=dt)
            V = (rdt(momentum) * st["momentum_buffer"] - np.conj(G).T).astype(dt)
            MX = V @ X
            XMX = X @ MX
            XXMX = np.conj(X).T @ XMX
            W_hat = (MX - rdt(0.5) * XXMX).astype(dt)
            W = (W_hat - np.conj(W_hat).T).astype(dt)
            t = rdt(0.5) * rdt(2) / (matrix_norm_one(W) + rdt(EPS))
            alpha = min(t, lr)
            I = np.eye(W.shape[0], dtype=dt)
            left = (I - rdt(alpha / 2) * W).astype(dt)
            right = (I + rdt(alpha / 2) * W).astype(dt)
            Y = np.linalg.inv(left) @ right @ np.conj(X).T           # compute_Y :66-74
            p_new = np.conj(Y).T
            st["momentum_buffer"] = (W @ np.conj(X).T).astype(dt)
            p[...] = p_new.reshape(size).astype(dt)
        else:
            d_p = g
            if weight_decay != 0:
                d_p += rdt(weight_decay) * p
            if momentum != 0:
                st = state.setdefault(i, {})
                if "momentum_buffer" not in st:
                    buf = st["momentum_buffer"] = d_p.copy()
                else:
                    buf = st["momentum_buffer"]
                    buf *= rdt(momentum)
                    buf += rdt(1 - dampening) * d_p
                d_p = d_p + rdt(momentum) * buf if nesterov else buf
            p -= rdt(lr) * d_p
