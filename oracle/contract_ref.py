"""ORACLE (test infrastructure only): a plain numpy pairwise einsum executor.

Restates what the reference's opt_einsum ContractExpression does at call time
(tneq_qc/contractor/einsum_strategy.py:622-643 -> opt_einsum.contract_expression(...)(*tensors)):
a sequence of pairwise tensordots, each = transpose -> reshape -> matmul, with the same
einsum semantics (a symbol shared by two operands and absent from the rest and the output is
summed; a symbol kept by the output or a later operand survives; batch symbols allowed).
The contraction ORDER only changes floating-point rounding, not the result; this oracle picks
pairs greedily by removed size (opt_einsum 'greedy' cost rule) and accumulates in complex128 /
float64 so it serves as the exact side of every tolerance check.
Symbols may be any unicode characters (get_symbol beyond 52 letters), unlike np.einsum.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def parse_equation(eq: str) -> Tuple[List[str], str]:
    if "->" in eq:
        lhs, rhs = eq.split("->")
    else:  # implicit output: symbols appearing exactly once, sorted (numpy/opt_einsum rule)
        lhs = eq
        cnt = {}
        for ch in lhs.replace(",", ""):
            cnt[ch] = cnt.get(ch, 0) + 1
        rhs = "".join(sorted(c for c, k in cnt.items() if k == 1))
    terms = lhs.split(",") if lhs != "" else []
    return terms, rhs


def _exact(a: np.ndarray) -> np.ndarray:
    return a.astype(np.complex128 if np.iscomplexobj(a) else np.float64, copy=False)


def sliced_operands(eq: str, arrays: Sequence[np.ndarray], sliced: Sequence[str], slice_id: int):
    """Operands of slice `slice_id` of a sliced contraction: every symbol in `sliced` is fixed to
    the digit of `slice_id` (row-major over `sliced`, last fastest — the enumeration of
    tq_plan_execute) and removed from the equation.  Returns (equation, operands)."""
    terms, rhs = parse_equation(eq)
    ext = {}
    for t, a in zip(terms, arrays):
        for c, e in zip(t, np.shape(a)):
            ext[c] = e
    idx, rem = {}, int(slice_id)
    for s in reversed(list(sliced)):
        idx[s] = rem % ext[s]
        rem //= ext[s]
    if rem:
        raise ValueError("slice id out of range")
    ops = []
    for t, a in zip(terms, arrays):
        ix = tuple(idx[c] if c in idx else slice(None) for c in t)
        ops.append(np.ascontiguousarray(np.asarray(a)[ix]))
    new_terms = ["".join(c for c in t if c not in idx) for t in terms]
    return ",".join(new_terms) + "->" + rhs, ops


def _sum_out(t: str, a: np.ndarray, keep: set) -> Tuple[str, np.ndarray]:
    axes = tuple(i for i, c in enumerate(t) if c not in keep)
    if axes:
        a = a.sum(axis=axes)
        t = "".join(c for c in t if c in keep)
    return t, a


def contract_pair(ta: str, a: np.ndarray, tb: str, b: np.ndarray, keep: set) -> Tuple[str, np.ndarray]:
    """One pairwise step: permute -> reshape -> matmul (the tensordot of the reference path)."""
    sa, sb = set(ta), set(tb)
    ta, a = _sum_out(ta, a, keep | sb)
    tb, b = _sum_out(tb, b, keep | sa)
    sa, sb = set(ta), set(tb)
    batch = [c for c in ta if c in sb and c in keep]
    contr = [c for c in ta if c in sb and c not in keep]
    fa = [c for c in ta if c not in sb]
    fb = [c for c in tb if c not in sa]
    ext = {c: a.shape[i] for i, c in enumerate(ta)}
    ext.update({c: b.shape[i] for i, c in enumerate(tb)})
    pa = [ta.index(c) for c in batch + fa + contr]
    pb = [tb.index(c) for c in batch + contr + fb]
    nb = int(np.prod([ext[c] for c in batch])) if batch else 1
    nm = int(np.prod([ext[c] for c in fa])) if fa else 1
    nk = int(np.prod([ext[c] for c in contr])) if contr else 1
    nn = int(np.prod([ext[c] for c in fb])) if fb else 1
    A = np.transpose(a, pa).reshape(nb, nm, nk)
    B = np.transpose(b, pb).reshape(nb, nk, nn)
    C = np.matmul(A, B)
    out_t = "".join(batch + fa + fb)
    return out_t, C.reshape([ext[c] for c in out_t])


def greedy_path(terms: Sequence[str], shapes: Sequence[Sequence[int]], rhs: str):
    """SSA path chosen by opt_einsum's greedy rule: contract the pair that removes the most
    size (result - a - b smallest), preferring pairs that share a symbol."""
    ext = {}
    for t, s in zip(terms, shapes):
        for c, e in zip(t, s):
            ext[c] = e
    live = {i: t for i, t in enumerate(terms)}
    nid = len(terms)
    path = []

    def size(t):
        return int(np.prod([ext[c] for c in t])) if t else 1

    while len(live) > 1:
        best = None
        ids = sorted(live)
        for x in range(len(ids)):
            for y in range(x + 1, len(ids)):
                i, j = ids[x], ids[y]
                ti, tj = live[i], live[j]
                shared = set(ti) & set(tj)
                others = set(rhs)
                for k, t in live.items():
                    if k != i and k != j:
                        others |= set(t)
                res = "".join(c for c in dict.fromkeys(ti + tj) if c in others)
                cost = (0 if shared else 1, size(res) - size(ti) - size(tj), i, j)
                if best is None or cost < best[0]:
                    best = (cost, i, j, res)
        _, i, j, res = best
        path.append((i, j))
        del live[i], live[j]
        live[nid] = res
        nid += 1
    return path


def contract(eq: str, *arrays: np.ndarray, path=None, exact: bool = True) -> np.ndarray:
    """Evaluate an einsum equation (unicode symbols allowed) in exact arithmetic (complex128 /
    float64), or with exact=False in the operands' own dtype (the CPU baseline's complex64 run:
    same plan, same dtype as the GPU path)."""
    terms, rhs = parse_equation(eq)
    if len(terms) != len(arrays):
        raise ValueError(f"equation has {len(terms)} operands, got {len(arrays)}")
    ext = {}
    for t, a in zip(terms, arrays):
        if len(t) != a.ndim:
            raise ValueError(f"term {t!r} does not match shape {a.shape}")
        for c, e in zip(t, a.shape):
            if ext.setdefault(c, e) != e:
                raise ValueError(f"symbol {c!r} has inconsistent extents")
    conv = _exact if exact else (lambda a: a)
    live = {i: (t, conv(np.asarray(a))) for i, (t, a) in enumerate(zip(terms, arrays))}
    if path is None:
        path = greedy_path(terms, [a.shape for a in arrays], rhs)
    nid = len(terms)
    for i, j in path:
        (ti, a), (tj, b) = live.pop(i), live.pop(j)
        keep = set(rhs)
        for t, _ in live.values():
            keep |= set(t)
        live[nid] = contract_pair(ti, a, tj, b, keep)
        nid += 1
    if len(live) != 1:
        raise ValueError("path does not reduce to one tensor")
    (t, a), = live.values()
    t, a = _sum_out(t, a, set(rhs))
    return np.transpose(a, [t.index(c) for c in rhs]) if rhs else a.reshape(())


def contract_sliced(eq: str, arrays: Sequence[np.ndarray], sliced: Sequence[str], path,
                    slice_ids=None, exact: bool = True) -> np.ndarray:
    """Sum over slices `slice_ids` (default: all) of contract(sliced_operands(eq, arrays, sliced,
    s), path=path) -- the quantity a sliced execute call accumulates (tq_plan_execute; the
    reference's partial contractions reduced by all_reduce(SUM), distributed_engine.py:1477-1497).
    Path steps that read no sliced input are evaluated once and reused by every slice (the
    result is the same as summing independent `contract` calls; only the work is shared)."""
    terms, rhs = parse_equation(eq)
    sl = set(sliced)
    ext = {}
    for t, a in zip(terms, arrays):
        for c, e in zip(t, np.shape(a)):
            ext[c] = e
    n_sl = int(np.prod([ext[s] for s in sliced])) if sliced else 1
    ids = range(n_sl) if slice_ids is None else slice_ids
    conv = _exact if exact else (lambda a: a)
    dep = {i: bool(set(t) & sl) for i, t in enumerate(terms)}
    tlive = {i: t for i, t in enumerate(terms)}
    nid = len(terms)
    for i, j in path:   # dependence of every SSA value on a sliced input
        dep[nid] = dep[i] or dep[j]
        nid += 1
    # slice-invariant SSA values, computed once (their terms hold no sliced symbol)
    inv = {i: (t, conv(np.asarray(a))) for i, (t, a) in enumerate(zip(terms, arrays)) if not dep[i]}
    live_t = dict(tlive)
    nid = len(terms)
    for i, j in path:
        ti, tj = live_t.pop(i), live_t.pop(j)
        if not dep[nid]:
            keep = set(rhs)
            for t in live_t.values():
                keep |= set(t)
            keep -= sl
            inv[nid] = contract_pair(ti, inv[i][1], tj, inv[j][1], keep)
            inv.pop(i)
            inv.pop(j)
        live_t[nid] = "".join(c for c in dict.fromkeys(ti + tj)) if dep[nid] else inv[nid][0]
        nid += 1
    total = None
    for s in ids:
        seq, sops = sliced_operands(eq, arrays, sliced, s)
        sterms, _ = parse_equation(seq)
        live = {i: (sterms[i], conv(sops[i])) for i in range(len(terms)) if dep[i]}
        live.update({k: v for k, v in inv.items()})
        nid = len(terms)
        for i, j in path:
            if dep[nid]:
                (ti, a), (tj, b) = live.pop(i), live.pop(j)
                keep = set(rhs)
                for t, _ in live.values():
                    keep |= set(t)
                live[nid] = contract_pair(ti, a, tj, b, keep)
            nid += 1
        (t, a), = live.values()
        t, a = _sum_out(t, a, set(rhs))
        r = np.transpose(a, [t.index(c) for c in rhs]) if rhs else a.reshape(())
        total = r.copy() if total is None else total + r
    return total
