"""Equation parsing, contraction-path finding and index slicing (host side of the engine).

The reference delegates all of this to opt_einsum (tneq_qc/contractor/einsum_strategy.py:622-643,
`optimize=Configuration.opt_einsum_optimize='greedy'`, tneq_qc/config.py:3; the workload uses
`optimize="auto"`, symmetry_breaking_quantum.py:142,154,213).  opt_einsum is an unpinned, absent
third-party dependency, so the build ships its own path finders:

  * ``greedy``  — opt_einsum's greedy rule (pick the connected pair whose contraction removes the
                  most size: size(out) - size(a) - size(b)), heap-driven, O(E log E);
  * ``linear``  — a sweep: grow one running tensor by absorbing, among the tensors connected to it,
                  the one that keeps it smallest (ties broken by an order hint, e.g. (qubit, time)).
                  For quantum circuits this yields the qubit-by-qubit sweep whose every step is a
                  small-operand absorption (the APPLY lowering of the plan compiler);
  * ``partition`` — a tree: sweep each group of a partition, then contract the group results
                  (e.g. the left/right halves of a circuit cut: the boundary GEMM);
and a slicer that removes contracted modes (index slicing).

The path only changes summation order (rounding), never the mathematical result; symbol
bookkeeping (which output axis is which) is preserved exactly.
"""
from __future__ import annotations

import heapq
import math
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple


def get_symbol(i: int) -> str:
    """opt_einsum.get_symbol semantics (used for core names and einsum symbols throughout the
    reference: qctn.py:498, einsum_strategy.py:162-182, greedy_strategy.py:414)."""
    if i < 52:
        return "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"[i]
    if i >= 55296:
        return chr(i + 2048)
    return chr(i + 140)


@dataclass
class Network:
    """An einsum as integer modes: terms[i] = mode ids of operand i, out = output mode ids."""
    terms: List[List[int]]
    out: List[int]
    extents: Dict[int, int]
    symbols: List[str] = field(default_factory=list)  # mode id -> original symbol

    def size(self, modes: Iterable[int]) -> int:
        p = 1
        for m in modes:
            p *= self.extents[m]
        return p


def parse_equation(eq: str, shapes: Sequence[Sequence[int]]) -> Network:
    """Parse "ab,bc->ac" (any unicode symbols, explicit or implicit output) into a Network."""
    eq = eq.replace(" ", "")
    if "->" in eq:
        lhs, rhs = eq.split("->")
        implicit = False
    else:
        lhs, rhs, implicit = eq, "", True
    terms_s = lhs.split(",") if lhs != "" else []
    if len(terms_s) != len(shapes):
        raise ValueError(f"einsum equation has {len(terms_s)} operands but {len(shapes)} shapes were given")
    if implicit:
        cnt: Dict[str, int] = {}
        for ch in lhs.replace(",", ""):
            cnt[ch] = cnt.get(ch, 0) + 1
        rhs = "".join(sorted(c for c, k in cnt.items() if k == 1))
    sym2id: Dict[str, int] = {}
    symbols: List[str] = []
    extents: Dict[int, int] = {}
    terms: List[List[int]] = []
    for t, shp in zip(terms_s, shapes):
        shp = tuple(int(x) for x in shp)
        if len(t) != len(shp):
            raise ValueError(f"term {t!r} has {len(t)} symbols but the operand has shape {shp}")
        ids = []
        for ch, e in zip(t, shp):
            if ch not in sym2id:
                sym2id[ch] = len(symbols)
                symbols.append(ch)
            m = sym2id[ch]
            if m in ids:
                raise ValueError(f"repeated symbol {ch!r} inside one operand (diagonals) is not supported")
            if extents.setdefault(m, e) != e:
                raise ValueError(f"symbol {ch!r} has inconsistent extents {extents[m]} vs {e}")
            ids.append(m)
        terms.append(ids)
    out = []
    for ch in rhs:
        if ch not in sym2id:
            raise ValueError(f"output symbol {ch!r} does not appear in any operand")
        if sym2id[ch] in out:
            raise ValueError(f"output symbol {ch!r} repeated")
        out.append(sym2id[ch])
    return Network(terms, out, extents, symbols)


# ---------------------------------------------------------------------------------------------
# path finders — all return an opt_einsum-style SSA path: list of (i, j); new id = n + step
# ---------------------------------------------------------------------------------------------

class _State:
    def __init__(self, net: Network):
        self.net = net
        self.live: Dict[int, Tuple[int, ...]] = {i: tuple(t) for i, t in enumerate(net.terms)}
        self.owners: Dict[int, set] = {}
        for i, t in self.live.items():
            for m in t:
                self.owners.setdefault(m, set()).add(i)
        self.outset = set(net.out)
        self.next_id = len(net.terms)

    def result(self, i: int, j: int) -> Tuple[int, ...]:
        ti, tj = self.live[i], self.live[j]
        res = []
        seen = set()
        for m in ti + tj:
            if m in seen:
                continue
            seen.add(m)
            own = self.owners[m]
            if m in self.outset or len(own - {i, j}) > 0:
                res.append(m)
        return tuple(res)

    def contract(self, i: int, j: int) -> int:
        res = self.result(i, j)
        for m in self.live[i] + self.live[j]:
            self.owners[m].discard(i)
            self.owners[m].discard(j)
        del self.live[i], self.live[j]
        k = self.next_id
        self.next_id += 1
        self.live[k] = res
        for m in res:
            self.owners.setdefault(m, set()).add(k)
        return k

    def neighbours(self, i: int) -> set:
        nb = set()
        for m in self.live[i]:
            nb |= self.owners[m]
        nb.discard(i)
        return nb


def greedy_path(net: Network) -> List[Tuple[int, int]]:
    """opt_einsum-style greedy: repeatedly contract the connected pair with the smallest
    size(result) - size(a) - size(b); disconnected leftovers are joined smallest-first."""
    st = _State(net)
    size = net.size
    heap: List[Tuple[int, int, int, int]] = []

    def push(i, j):
        if i > j:
            i, j = j, i
        c = size(st.result(i, j)) - size(st.live[i]) - size(st.live[j])
        heapq.heappush(heap, (c, i, j, 0))

    for i in list(st.live):
        for j in st.neighbours(i):
            if i < j:
                push(i, j)
    path = []
    while len(st.live) > 1:
        while heap and (heap[0][1] not in st.live or heap[0][2] not in st.live):
            heapq.heappop(heap)
        if heap:
            _, i, j, _ = heapq.heappop(heap)
        else:  # no connected pair: outer-product the two smallest tensors
            ids = sorted(st.live, key=lambda t: (size(st.live[t]), t))
            i, j = ids[0], ids[1]
        path.append((i, j))
        k = st.contract(i, j)
        for nb in st.neighbours(k):
            push(k, nb)
    return path


def vector_absorptions(net: Network) -> List[Tuple[int, int]]:
    """Pre-contraction pairs (vector, neighbour) for every rank-1 operand whose single contracted
    mode is shared with exactly one other operand: product-state inputs and output projectors are
    folded into their gate before any sweep, so no sweep step ever grows the running tensor by a
    leg that a vector removes one step later.  A neighbour keeps at least one leg (never becomes
    a scalar); several vectors on one gate are absorbed one after the other."""
    owners: Dict[int, List[int]] = {}
    for i, t in enumerate(net.terms):
        for m in t:
            owners.setdefault(m, []).append(i)
    outset = set(net.out)
    legs = {i: len(t) for i, t in enumerate(net.terms)}
    pre = []
    for i, t in enumerate(net.terms):
        if len(t) != 1 or t[0] in outset:
            continue
        own = [j for j in owners[t[0]] if j != i]
        if len(own) != 1 or len(net.terms[own[0]]) < 2 or legs[own[0]] <= 1:
            continue
        legs[own[0]] -= 1
        pre.append((i, own[0]))
    return pre


def _apply_pre(st: "_State", pre: Sequence[Tuple[int, int]]):
    """Contract the (original-id) pairs of `pre` on `st`; returns (path, alias original->live id)."""
    alias: Dict[int, int] = {}
    find = lambda x: alias.get(x, x) if alias.get(x, x) == x else find(alias[x])
    path = []
    for a, b in pre:
        ia, ib = find(a), find(b)
        path.append((ia, ib))
        k = st.contract(ia, ib)
        alias[ia] = k
        alias[ib] = k
        alias[k] = k
    return path, find


def _alias_group(ids: Sequence[int], find, rank_of: Dict[int, int]):
    """Map original ids (and an order rank) onto the live ids after pre-contraction."""
    out: List[int] = []
    rank: Dict[int, int] = {}
    for t in ids:
        k = find(t)
        if k not in rank:
            out.append(k)
            rank[k] = rank_of.get(t, len(rank_of) + t)
        else:
            rank[k] = min(rank[k], rank_of.get(t, len(rank_of) + t))
    return out, rank


def linear_path(net: Network, order: Optional[Sequence[int]] = None,
                subset: Optional[Sequence[int]] = None,
                pre: Sequence[Tuple[int, int]] = ()) -> Tuple[List[Tuple[int, int]], int]:
    """Sweep path over `subset` (default: all operands): start from the first tensor of the order
    hint and repeatedly absorb the connected tensor that keeps the running tensor smallest
    (ties: earliest in the order hint).  `pre` = original-id pairs contracted first (e.g.
    vector_absorptions).  Returns (path over the full SSA numbering, final id).
    Only tensors of `subset` are touched; the caller continues the numbering."""
    ids = list(range(len(net.terms))) if subset is None else list(subset)
    if order is None:
        order = ids
    rank = {t: k for k, t in enumerate(order)}
    for t in ids:
        rank.setdefault(t, len(rank) + t)
    st = _State(net)
    path, find = _apply_pre(st, pre)
    ids, rank = _alias_group(ids, find, rank)
    p, root = _linear_on_state(st, ids, rank)
    return path + p, root


def _linear_on_state(st: _State, ids: Sequence[int], rank: Dict[int, int], strict: bool = False):
    """strict: absorb in the order hint's order (connected tensors first), no size rule."""
    size = st.net.size
    remaining = set(ids)
    first = min(remaining, key=lambda t: rank[t])
    remaining.discard(first)
    cur = first
    path = []
    while remaining:
        cand = st.neighbours(cur) & remaining
        if not cand:
            nxt = min(remaining, key=lambda t: rank[t])
        elif strict:
            nxt = min(cand, key=lambda t: rank[t])
        else:
            nxt = min(cand, key=lambda t: (size(st.result(cur, t)), rank[t]))
        remaining.discard(nxt)
        path.append((cur, nxt))
        cur = st.contract(cur, nxt)
    return path, cur


def partition_path(net: Network, groups: Sequence[Sequence[int]],
                   orders: Optional[Sequence[Sequence[int]]] = None,
                   pre: Sequence[Tuple[int, int]] = (), strict: bool = False,
                   defer: Optional[Sequence[int]] = None) -> List[Tuple[int, int]]:
    """Sweep each group with linear_path, then contract the group results left to right.
    `pre` pairs (original ids, both in one group) are contracted before the sweeps; `strict`
    follows each order hint exactly (see _linear_on_state).

    `defer[g]` = the number of tensors at the END of group g's sweep that are not absorbed into
    the group result but into the contracted boundary afterwards (greedily, smallest result first).
    A sweep's last tensors are the gates that grow it into the boundary operand -- they add the
    open legs and the cut legs the other side contracts -- so absorbing them after the boundary
    contraction shrinks that contraction by orders of magnitude (C4: the 2^36-MAC boundary GEMM
    per slice becomes a 2^31-MAC one over the cut legs those gates do not touch; deferred_search
    picks the counts by the path cost model)."""
    st = _State(net)
    path, find = _apply_pre(st, pre)
    roots = []
    later: List[int] = []
    for g, grp in enumerate(groups):
        order = orders[g] if orders is not None else list(grp)
        rank0 = {t: k for k, t in enumerate(order)}
        ids, rank = _alias_group(list(grp), find, rank0)
        t = int(defer[g]) if defer is not None and g < len(defer) else 0
        if t > 0:
            # the sweep's absorption order on a scratch state, then the sweep without its tail
            seq = _sweep_sequence(st, ids, rank, strict)
            t = min(t, len(seq) - 1)
            keep, tail = seq[:len(seq) - t], seq[len(seq) - t:]
            cur = keep[0]
            for nxt in keep[1:]:
                path.append((cur, nxt))
                cur = st.contract(cur, nxt)
            roots.append(cur)
            later += tail
            continue
        p, root = _linear_on_state(st, ids, rank, strict)
        path += p
        roots.append(root)
    cur = roots[0]
    for r in roots[1:]:
        path.append((cur, r))
        cur = st.contract(cur, r)
    rem = set(later)
    size = st.net.size
    while rem:
        cand = st.neighbours(cur) & rem or rem
        nxt = min(cand, key=lambda t: (size(st.result(cur, t)), t))
        rem.discard(nxt)
        path.append((cur, nxt))
        cur = st.contract(cur, nxt)
    return path


def _sweep_sequence(st: "_State", ids: Sequence[int], rank: Dict[int, int], strict: bool) -> List[int]:
    """The order in which _linear_on_state would absorb `ids` (first tensor first), computed on
    a copy of the state."""
    import copy
    sc = copy.deepcopy(st)
    size = sc.net.size
    remaining = set(ids)
    first = min(remaining, key=lambda t: rank[t])
    remaining.discard(first)
    cur, seq = first, [first]
    while remaining:
        cand = sc.neighbours(cur) & remaining
        if not cand:
            nxt = min(remaining, key=lambda t: rank[t])
        elif strict:
            nxt = min(cand, key=lambda t: rank[t])
        else:
            nxt = min(cand, key=lambda t: (size(sc.result(cur, t)), rank[t]))
        remaining.discard(nxt)
        seq.append(nxt)
        cur = sc.contract(cur, nxt)
    return seq


def deferred_search(net: Network, groups: Sequence[Sequence[int]], orders, pre, removed=(),
                    max_defer: int = 32, step: int = 2) -> Tuple[int, int]:
    """(defer_left, defer_right) of two-group partition_path minimising the cost model's estimate
    of an execute (path_info.est_seconds; `removed` = the sliced modes it is priced with)."""
    best = None
    for tl in range(0, max_defer + 1, step):
        for tr in range(0, max_defer + 1, step):
            try:
                p = partition_path(net, groups, orders, pre=pre, defer=(tl, tr))
                info = path_info(net, p, removed)
            except ValueError:
                continue
            key = (info.est_seconds, info.max_size, tl + tr)
            if best is None or key < best[0]:
                best = (key, (tl, tr))
    return best[1] if best else (0, 0)


@dataclass
class PathInfo:
    flops: float            # complex-MAC count of a full execute (sum over steps of the product
                            # of all extents involved; sliced steps counted once per slice)
    max_size: int           # largest intermediate (elements)
    steps: List[Tuple[int, int, Tuple[int, ...], float]]  # (i, j, result modes, macs per run)
    once_flops: float = 0.0   # slice-invariant part (hoisted by the plan executor)
    slice_flops: float = 0.0  # per-slice part
    n_slices: int = 1
    est_seconds: float = 0.0  # roofline estimate of a full execute on one MI355X
    t_once: float = 0.0       # its slice-invariant part (replicated on every rank)
    t_slice: float = 0.0      # its per-slice part (one slice)

    def est_ranks(self, world: int) -> float:
        """Estimate of one rank's share when the slices are split over `world` ranks."""
        return self.t_once + self.t_slice * -(-self.n_slices // max(1, world))


# roofline constants for the cost model (MI355X: ~5 TB/s achievable HBM, ~110 TF/s sustained
# fp32-MFMA GEMM); only ratios matter for path / slice choices
_BW, _PEAK, _ESZ, _FPM = 5.0e12, 1.1e14, 8.0, 8.0


def path_info(net: Network, path: Sequence[Tuple[int, int]], removed: Iterable[int] = ()) -> PathInfo:
    """Cost of a path; modes in `removed` (sliced) count with extent 1.  Steps that touch no
    sliced input are slice-invariant: the native plan hoists them out of the slice loop."""
    removed = set(removed)
    ext = {m: (1 if m in removed else e) for m, e in net.extents.items()}
    st = _State(net)
    size = lambda ms: math.prod(ext[m] for m in ms)
    dep = {i: any(m in removed for m in t) for i, t in st.live.items()}
    n_sl = math.prod(net.extents[m] for m in removed) if removed else 1
    once = per = t_once = t_per = 0.0
    mx = max([size(t) for t in st.live.values()] + [1])
    steps = []
    for i, j in path:
        if i not in st.live or j not in st.live:
            raise ValueError(f"invalid path step ({i}, {j})")
        union = set(st.live[i]) | set(st.live[j])
        macs = float(size(union))
        si, sj = size(st.live[i]), size(st.live[j])
        k = st.contract(i, j)
        dep[k] = dep[i] or dep[j]
        sk = size(st.live[k])
        t = max((si + sj + sk) * _ESZ / _BW, macs * _FPM / _PEAK) + 2e-6  # + launch
        if dep[k]:
            per += macs
            t_per += t
        else:
            once += macs
            t_once += t
        mx = max(mx, sk)
        steps.append((i, j, st.live[k], macs))
    if len(st.live) != 1:
        raise ValueError("path does not contract the network to one tensor")
    return PathInfo(once + per * n_sl, mx, steps, once, per, n_sl, t_once + t_per * n_sl, t_once, t_per)


def validate_path(n_terms: int, path: Sequence[Tuple[int, int]]) -> None:
    used = set()
    for s, (i, j) in enumerate(path):
        nid = n_terms + s
        for x in (i, j):
            if not (0 <= x < nid) or x in used:
                raise ValueError(f"invalid path step {s}: ({i}, {j})")
            used.add(x)
        if i == j:
            raise ValueError(f"invalid path step {s}: ({i}, {j})")
    if len(path) != max(0, n_terms - 1):
        raise ValueError(f"a pairwise path needs {n_terms - 1} steps, got {len(path)}")


def choose_slices(net: Network, path: Sequence[Tuple[int, int]], n_modes: int,
                  candidates: Optional[Sequence[int]] = None) -> List[int]:
    """Greedy index slicing: repeatedly fix the contracted mode whose removal minimises the
    roofline time of an execute = hoisted slice-invariant steps + slices x per-slice steps, on
    one GPU plus on one rank of an 8-GPU split (the hoisted part is replicated on every rank, so
    among equally cheap single-GPU choices the one with the smaller hoisted part wins).
    Output modes are never sliced."""
    outset = set(net.out)
    if candidates is None:
        candidates = [m for m in net.extents if m not in outset]
    chosen: List[int] = []
    for _ in range(n_modes):
        best = None
        for m in candidates:
            if m in chosen or m in outset:
                continue
            info = path_info(net, path, chosen + [m])
            key = (info.est_seconds + info.est_ranks(8), info.max_size, m)
            if best is None or key < best[0]:
                best = (key, m)
        if best is None:
            break
        chosen.append(best[1])
    return chosen
