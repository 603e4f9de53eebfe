"""Symbolic replay of GreedyStrategy's compute_fn: the reference's qubit-group sweep, run on
axis *labels* instead of tensors, folded into ONE flat einsum for the HIP tree executor.

The reference (tneq_qc/contractor/greedy_strategy.py:41-1080) contracts the L·M·R network group
by group with torch.einsum, and its bookkeeping has behaviour that a hand-written sandwich
equation does not reproduce:
  * qubits without a circuit state or Mx leave legs open, in the order the groups produce them
    (:105-223, :864-880) — and _contract_remaining sums every non-batch leg it sees (:1030-1078);
  * right_qctn=QCTN registers its cores under core_idx + len(left cores) (:224-256) but step 2.2
    looks neighbours up by the right QCTN's own indices (:352-399), so right-core bonds keep
    stale neighbour pointers: they never share a symbol, become "internal" to whatever group the
    stale pointer lands in, and are summed there; the axes are read through the dim map of
    :764-822 with `original_in_edge_count` never set.
Replaying the same steps on labels gives the reference's result exactly, whatever the inputs:
every group einsum becomes a relabelling (a union of the labels its equation identifies), and a
chain of einsums is one einsum over all leaf operands (products of sums = sum of products), which
the native plan then contracts along its own path.  No arithmetic happens here.

Leaf operands (the recipe): ('L', core) the core as given, ('R', core) conj(core) for complex
cores (`_get_tensor` 'transpose', :675-681), ('Rq', core) a right_qctn core as given,
('S', q) circuit state of qubit q, ('M', q) Mx of qubit q.
"""
from __future__ import annotations

from copy import deepcopy
from typing import Dict, List, Optional, Sequence, Tuple

from ..einsum import get_symbol

LEFT, MIDDLE, RIGHT = "left", "middle", "right"


class _Labels:
    """Union-find over global axis labels."""

    def __init__(self):
        self.parent: List[int] = []

    def new(self) -> int:
        self.parent.append(len(self.parent))
        return len(self.parent) - 1

    def find(self, x: int) -> int:
        p = self.parent
        while p[x] != x:
            p[x] = p[p[x]]
            x = p[x]
        return x

    def union(self, a: int, b: int):
        a, b = self.find(a), self.find(b)
        if a != b:
            self.parent[a] = b


class _Sym:
    """A symbolic tensor: the product of `leaves` (leaf key, label per axis) with open axes `axes`
    (everything else summed)."""
    __slots__ = ("leaves", "axes")

    def __init__(self, leaves, axes):
        self.leaves = leaves
        self.axes = axes

    @property
    def ndim(self) -> int:
        return len(self.axes)


class _Replay:
    def __init__(self, leaf_ndim: Dict[tuple, int]):
        self.lab = _Labels()
        self.leaf_ndim = leaf_ndim

    def leaf(self, key) -> _Sym:
        ax = [self.lab.new() for _ in range(self.leaf_ndim[key])]
        return _Sym([(key, list(ax))], list(ax))

    def einsum(self, parts: Sequence[str], out: str, syms: Sequence[_Sym]) -> _Sym:
        """torch.einsum(",".join(parts) + "->" + out, *syms) on labels."""
        cmap: Dict[str, int] = {}
        for p, s in zip(parts, syms):
            if len(p) != s.ndim:
                raise RuntimeError(f"einsum(): the number of subscripts in the equation ({len(p)}) "
                                   f"does not match the number of dimensions ({s.ndim})")
            for c, g in zip(p, s.axes):
                if c in cmap:
                    self.lab.union(cmap[c], g)
                else:
                    cmap[c] = g
        if len(set(out)) != len(out):
            raise RuntimeError("einsum(): output subscript appears more than once")
        for c in out:
            if c not in cmap:
                raise RuntimeError(f"einsum(): output subscript {c} does not appear in the inputs")
        leaves = [lf for s in syms for lf in s.leaves]
        return _Sym(leaves, [cmap[c] for c in out])

    def flat(self, s: _Sym) -> Tuple[str, List[tuple]]:
        sym: Dict[int, str] = {}

        def name(g):
            r = self.lab.find(g)
            if r not in sym:
                sym[r] = get_symbol(len(sym))
            return sym[r]

        terms = ["".join(name(g) for g in ax) for _, ax in s.leaves]
        for t in terms:
            if len(set(t)) != len(t):
                raise NotImplementedError("greedy replay produced a diagonal (repeated index) operand")
        out = "".join(name(g) for g in s.axes)
        return ",".join(terms) + "->" + out, [k for k, _ in s.leaves]


def _present(container, q) -> bool:
    """greedy_strategy.py:82-99 / :141-156: dict -> key present, list/tuple -> index in range."""
    if container is None:
        return False
    if isinstance(container, dict):
        return q in container
    if isinstance(container, (list, tuple)):
        return q < len(container)
    return True


def greedy_equation(qctn, state_dims: Dict[int, int], mx_ndims: Dict[int, Tuple[int, int, int]],
                    core_ndims: Dict[str, int], right_qctn="symmetric",
                    right_core_ndims: Optional[Dict[str, int]] = None) -> Tuple[str, List[tuple]]:
    """Flat einsum (equation, leaf recipe) equal to GreedyStrategy's compute_fn result.

    state_dims: qubit -> len(state) for every qubit the reference would attach a state to;
    mx_ndims:   qubit -> (ndim, dim[-2], dim[-1]) for every attached Mx (None entries excluded);
    core_ndims: core name -> ndim of the core tensor (same for right_core_ndims)."""
    from ..core.qctn import QCTN
    leaf_ndim: Dict[tuple, int] = {}
    for c, nd in core_ndims.items():
        leaf_ndim[("L", c)] = nd
        leaf_ndim[("R", c)] = nd
    for c, nd in (right_core_ndims or {}).items():
        leaf_ndim[("Rq", c)] = nd
    for q in state_dims:
        leaf_ndim[("S", q)] = 1
    for q, (nd, _, _) in mx_ndims.items():
        leaf_ndim[("M", q)] = nd
    R = _Replay(leaf_ndim)

    # ---- step 1: L cores, L states, Mx, R cores, R states (greedy_strategy.py:73-295)
    ents: List[dict] = []
    lmap: Dict[int, int] = {}
    for info in qctn.adjacency_table:
        lmap[info["core_idx"]] = len(ents)
        ents.append({"core_idx": len(ents), "src": ("L", info["core_name"]), "side": LEFT, "batch": "",
                     "in": deepcopy(info["in_edge_list"]), "out": deepcopy(info["out_edge_list"])})
    lstate: Dict[int, int] = {}
    for q in qctn.qubit_indices:
        if q in state_dims:
            lstate[q] = len(ents)
            ents.append({"core_idx": len(ents), "src": ("S", q), "side": LEFT, "batch": "", "in": [],
                         "out": [{"neighbor_idx": -1, "qubit_idx": q, "edge_rank": state_dims[q]}]})
    mxmap: Dict[int, int] = {}
    for q in qctn.qubit_indices:
        if q in mx_ndims:
            nd, d2, d1 = mx_ndims[q]
            mxmap[q] = len(ents)
            ents.append({"core_idx": len(ents), "src": ("M", q), "side": MIDDLE,
                         "batch": {3: "a", 4: "ab"}.get(nd, ""),
                         "in": [{"neighbor_idx": -1, "qubit_idx": q, "edge_rank": d2}],
                         "out": [{"neighbor_idx": -1, "qubit_idx": q, "edge_rank": d1}]})
    rmap: Dict[int, int] = {}
    if isinstance(right_qctn, str) and right_qctn == "symmetric":
        for info in qctn.adjacency_table:
            rmap[info["core_idx"]] = len(ents)
            ents.append({"core_idx": len(ents), "src": ("R", info["core_name"]), "side": RIGHT, "batch": "",
                         "in": deepcopy(info["out_edge_list"])[::-1],
                         "out": deepcopy(info["in_edge_list"])[::-1]})
    elif isinstance(right_qctn, QCTN) or hasattr(right_qctn, "adjacency_table"):
        for info in right_qctn.adjacency_table:
            # registered under the offset index, looked up below by the right QCTN's own indices
            rmap[info["core_idx"] + len(lmap)] = len(ents)
            ents.append({"core_idx": len(ents), "src": ("Rq", info["core_name"]), "side": RIGHT, "batch": "",
                         "in": deepcopy(info["in_edge_list"]), "out": deepcopy(info["out_edge_list"])})
    elif right_qctn is not None:
        raise ValueError("Invalid right_qctn parameter.")
    rstate: Dict[int, int] = {}
    for q in qctn.qubit_indices:
        if q in state_dims:
            rstate[q] = len(ents)
            ents.append({"core_idx": len(ents), "src": ("S", q), "side": RIGHT, "batch": "", "out": [],
                         "in": [{"neighbor_idx": -1, "qubit_idx": q, "edge_rank": state_dims[q]}]})

    # ---- step 2: wiring (:300-399)
    def wire(cmap, open_in, open_out, own):
        for uid in cmap.values():
            e = ents[uid]
            for kind, opened in (("in", open_in), ("out", open_out)):
                for ed in e[kind]:
                    if ed["neighbor_idx"] == -1:
                        q = ed["qubit_idx"]
                        if q in opened[0]:
                            v = opened[0][q]
                            ed["neighbor_idx"] = v
                            ents[v][opened[1]][0]["neighbor_idx"] = uid
                    elif ed["neighbor_idx"] in own:
                        ed["neighbor_idx"] = own[ed["neighbor_idx"]]

    wire(lmap, (lstate, "out"), (mxmap, "in"), lmap)
    wire(rmap, (mxmap, "out"), (rstate, "in"), rmap)

    # ---- step 2.5: symbols, 'a' and 'b' skipped (:404-449); out-edges first, propagated to the
    # neighbour's matching in-edge, then the in-edges still without one
    counter = [0]

    def next_symbol():
        while True:
            s = get_symbol(counter[0])
            counter[0] += 1
            if s not in ("a", "b"):
                return s

    for e in ents:
        for ed in e["out"]:
            if "symbol" in ed:
                continue
            ed["symbol"] = next_symbol()
            nb = ed["neighbor_idx"]
            if nb >= 0:
                for ie in ents[nb]["in"]:
                    if ie["neighbor_idx"] == e["core_idx"] and ie["qubit_idx"] == ed["qubit_idx"]:
                        ie["symbol"] = ed["symbol"]
                        break
    for e in ents:
        for ed in e["in"]:
            if "symbol" not in ed:
                ed["symbol"] = next_symbol()

    # ---- step 3: per qubit, groups of entries touching it, each contracted (:457-585)
    def tensor_of(e) -> _Sym:
        return e["sym"] if "sym" in e else R.leaf(e["src"])

    def right_dims(e, ndim):
        """axis symbols of a RIGHT entry through the reference's dim map (:757-810)."""
        n_in, n_out = len(e["out"]), len(e["in"])
        dims: List[Optional[str]] = [None] * ndim
        for k, ed in enumerate(e["out"]):
            dims[n_in - 1 - k] = ed["symbol"]
        for k, ed in enumerate(e["in"]):
            dims[n_in + n_out - 1 - k] = ed["symbol"]
        return dims

    def contract_group(group, q):
        if len(group) == 1 and not any(ed["qubit_idx"] == q for ed in group[0]["in"] + group[0]["out"]):
            return None
        ids = {e["core_idx"] for e in group}
        cin, cout, parts, syms, batch = [], [], [], [], set()

        def kept(ed):
            nb = ed["neighbor_idx"]
            internal = nb >= 0 and nb in ids
            return nb == -1 or (not internal and ed["qubit_idx"] != q)

        for e in group:
            t = tensor_of(e)
            syms.append(t)
            batch |= set(e["batch"])
            if e["side"] == RIGHT:
                body = "".join(s for s in right_dims(e, t.ndim - len(e["batch"])) if s is not None)
                cout += [dict(ed) for ed in e["out"] if kept(ed)]
                cin += [dict(ed) for ed in e["in"] if kept(ed)]
            else:
                body = "".join(ed["symbol"] for ed in e["in"]) + "".join(ed["symbol"] for ed in e["out"])
                cin += [dict(ed) for ed in e["in"] if kept(ed)]
                cout += [dict(ed) for ed in e["out"] if kept(ed)]
            parts.append(e["batch"] + body)
        nb = ("a" if "a" in batch else "") + ("b" if "b" in batch else "")
        out = nb + "".join(ed["symbol"] for ed in cin) + "".join(ed["symbol"] for ed in cout)
        return {"core_idx": -1, "sym": R.einsum(parts, out, syms), "side": MIDDLE, "batch": nb,
                "in": cin, "out": cout}

    def groups_of(entries):
        if len(entries) == 1:
            return [entries]
        pos = {e["core_idx"]: i for i, e in enumerate(entries)}
        uf = _Labels()
        for _ in entries:
            uf.new()
        for i, e in enumerate(entries):
            for ed in e["out"] + e["in"]:
                nb = ed["neighbor_idx"]
                if nb >= 0 and nb in pos:
                    uf.union(i, pos[nb])
        out: Dict[int, list] = {}
        for i, e in enumerate(entries):
            out.setdefault(uf.find(i), []).append(e)
        return list(out.values())

    next_uid = len(ents)
    for q in qctn.qubit_indices:
        on_q = [e for e in ents if any(ed["qubit_idx"] == q for ed in e["in"] + e["out"])]
        if not on_q:
            continue
        by_idx = {}
        for e in ents:
            by_idx.setdefault(e["core_idx"], e)
        extra = []
        for e in on_q:
            for ed in e["in"] + e["out"]:
                nb = ed["neighbor_idx"]
                if nb >= 0:
                    c = by_idx.get(nb)
                    if c is not None and c["src"] is not None and c["src"][0] == "S" and \
                            not any(c is x for x in on_q) and not any(c is x for x in extra):
                        extra.append(c)
        on_q += extra
        new, drop, remap = [], set(), {}
        for grp in groups_of(on_q):
            ne = contract_group(grp, q)
            if ne is None:
                continue
            ne["core_idx"] = next_uid
            ne["src"] = None
            next_uid += 1
            new.append(ne)
            for m in grp:
                drop.add(m["core_idx"])
                remap[m["core_idx"]] = ne["core_idx"]
        if not new:
            continue
        ents = [e for e in ents if e["core_idx"] not in drop] + new
        for e in ents:
            for ed in e["in"] + e["out"]:
                if ed["neighbor_idx"] in remap:
                    ed["neighbor_idx"] = remap[ed["neighbor_idx"]]

    # ---- step 4 (:596-606, :993-1080)
    if not ents:
        raise RuntimeError("No tensor left after contraction")
    if len(ents) == 1:
        return R.flat(tensor_of(ents[0]))
    parts, syms, outs = [], [], []
    for e in ents:
        t = tensor_of(e)
        syms.append(t)
        if e["side"] == MIDDLE:
            bd = t.ndim - 2
            p = ("a" if bd >= 1 else "") + ("b" if bd >= 2 else "")
            p += e["in"][0]["symbol"] if e["in"] else ""
            p += e["out"][0]["symbol"] if e["out"] else ""
        elif e["side"] == RIGHT:
            p = "".join(s for s in right_dims(e, t.ndim) if s is not None)
        else:
            p = "".join(ed["symbol"] for ed in e["in"]) + "".join(ed["symbol"] for ed in e["out"])
        parts.append(p)
        for b in "ab":
            if b in p and b not in outs:
                outs.append(b)
    return R.flat(R.einsum(parts, "".join(outs), syms))
