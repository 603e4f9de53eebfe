"""ORACLE (test infrastructure only): QCTN graph bookkeeping restated from the reference.

Follows, line by line in behaviour:
  get_symbol                      opt_einsum.get_symbol (published rule)
  QCTNRef.__init__ core order     tneq_qc/core/qctn.py:490-518
  QCTNRef._circuit_to_adjacency   tneq_qc/core/qctn.py:591-722
  core shapes                     tneq_qc/core/qctn.py:724-760 (input_shape + output_shape)
  build_core_only_expression      tneq_qc/contractor/einsum_strategy.py:136-194
  build_with_inputs_expression    tneq_qc/contractor/einsum_strategy.py:196-256
  build_with_vector_inputs_expression  einsum_strategy.py:258-318
  build_with_qctn_expression      einsum_strategy.py:320-416
  incidence_to_graph / build_brick_wall_IM   symmetry_breaking_quantum.py:15-63, 107-125
  split / merge (graph level)     tneq_qc/core/qctn.py:1217-1290, 1296-1506
"""
from __future__ import annotations

import re

import numpy as np

_BASE = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"


def get_symbol(i: int) -> str:
    """opt_einsum.get_symbol: 52 ASCII letters, then chr(i+140), skipping the surrogate block."""
    if i < 52:
        return _BASE[i]
    if i >= 55296:
        return chr(i + 2048)
    return chr(i + 140)


_IDX2CORE = [get_symbol(i) for i in range(10000)]          # qctn.py:498
_CORE2IDX = {c: i for i, c in enumerate(_IDX2CORE)}       # qctn.py:499
_FULL = set(_IDX2CORE)                                      # qctn.py:501


class QCTNRef:
    """Graph-only restatement of tneq_qc.core.qctn.QCTN (no backend, no weights)."""

    def __init__(self, graph: str):
        self.qubits = graph.strip().splitlines()                      # qctn.py:490
        self.nqubits = len(self.qubits)
        self.qubit_indices = list(range(self.nqubits))
        self.graph = graph
        self.cores = list(set(c for c in graph if c in _FULL))        # qctn.py:504
        self.cores.sort(key=lambda x: _CORE2IDX[x])                   # qctn.py:506
        self.ncores = len(self.cores)
        self._circuit_to_adjacency()

    def _circuit_to_adjacency(self):                                  # qctn.py:591-722
        cores = "".join(self.cores)
        d = {c: i for i, c in enumerate(self.cores)}
        self.dict_core2idx = d
        self.adjacency_table = [
            {"core_idx": i, "core_name": c, "in_edge_list": [], "out_edge_list": [],
             "input_shape": [], "output_shape": [], "input_dim": 1, "output_dim": 1}
            for i, c in enumerate(self.cores)
        ]
        inp = re.compile(rf"^(\d+)([{cores}])")
        outp = re.compile(rf"([{cores}])(\d+)$")
        conn = re.compile(rf"([{cores}])(\d+)(?=[{cores}])")
        for q, line in enumerate(self.qubits):
            line = line.strip().replace("-", "")
            in_rank, in_core = inp.match(line).groups()
            out_core, out_rank = outp.search(line).groups()
            self.adjacency_table[d[in_core]]["in_edge_list"].append(
                {"neighbor_idx": -1, "neighbor_name": "", "edge_rank": int(in_rank), "qubit_idx": q})
            self.adjacency_table[d[out_core]]["out_edge_list"].append(
                {"neighbor_idx": -1, "neighbor_name": "", "edge_rank": int(out_rank), "qubit_idx": q})
            for m in conn.finditer(line):
                end = m.end()
                if end >= len(line):
                    break
                c1, r1 = m.groups()
                c2 = line[end]
                self.adjacency_table[d[c1]]["out_edge_list"].append(
                    {"neighbor_idx": d[c2], "neighbor_name": c2, "edge_rank": int(r1), "qubit_idx": q})
                self.adjacency_table[d[c2]]["in_edge_list"].append(
                    {"neighbor_idx": d[c1], "neighbor_name": c1, "edge_rank": int(r1), "qubit_idx": q})
        for info in self.adjacency_table:
            info["input_shape"] = [e["edge_rank"] for e in info["in_edge_list"]]
            info["output_shape"] = [e["edge_rank"] for e in info["out_edge_list"]]
            info["input_dim"] = int(np.prod(info["input_shape"])) if info["input_shape"] else 1
            info["output_dim"] = int(np.prod(info["output_shape"])) if info["output_shape"] else 1
        # circuit tuple: (input ranks per core, adjacency matrix, output ranks per core) qctn.py:695-714
        self.circuit_inputs = [list(t["input_shape"]) for t in self.adjacency_table]
        self.circuit_outputs = [list(t["output_shape"]) for t in self.adjacency_table]

    def core_shape(self, name: str):
        t = self.adjacency_table[self.dict_core2idx[name]]
        return tuple(t["input_shape"] + t["output_shape"])            # qctn.py:754

    def core_shapes(self):
        return [self.core_shape(c) for c in self.cores]


def _edge_key(a, b, q):
    return tuple(sorted([a, b])) + (q,)


def _core_terms(qctn, on_input, on_output):
    """Shared walk of einsum_strategy.py:155-187 (symbol per internal edge, in/out hooks)."""
    sid = [0]
    emap = {}

    def fresh():
        s = get_symbol(sid[0])
        sid[0] += 1
        return s

    terms = []
    for info in qctn.adjacency_table:
        ci = info["core_idx"]
        t = ""
        for e in info["in_edge_list"]:
            if e["neighbor_idx"] == -1:
                s = fresh()
                on_input(s)
            else:
                k = _edge_key(e["neighbor_idx"], ci, e["qubit_idx"])
                if k not in emap:
                    emap[k] = fresh()
                s = emap[k]
            t += s
        for e in info["out_edge_list"]:
            if e["neighbor_idx"] == -1:
                s = fresh()
                on_output(s)
            else:
                k = _edge_key(ci, e["neighbor_idx"], e["qubit_idx"])
                if k not in emap:
                    emap[k] = fresh()
                s = emap[k]
            t += s
        terms.append(t)
    return terms, sid[0], emap


def build_core_only_expression(qctn):                                 # einsum_strategy.py:136-194
    rhs = []
    terms, _, _ = _core_terms(qctn, rhs.append, rhs.append)
    return ",".join(terms) + "->" + "".join(rhs), qctn.core_shapes()


def build_with_inputs_expression(qctn, inputs_shape):                 # einsum_strategy.py:196-256
    ins, rhs = [], []
    terms, _, _ = _core_terms(qctn, ins.append, rhs.append)
    return "".join(ins) + "," + ",".join(terms) + "->" + "".join(rhs), [tuple(inputs_shape)] + qctn.core_shapes()


def build_with_vector_inputs_expression(qctn, inputs_shapes):         # einsum_strategy.py:258-318
    ins, rhs = [], []
    terms, _, _ = _core_terms(qctn, ins.append, rhs.append)
    lhs = "".join(s + "," for s in ins) + ",".join(terms)
    return lhs + "->" + "".join(rhs), [tuple(s) for s in inputs_shapes] + qctn.core_shapes()


def build_with_qctn_expression(qctn, target):                         # einsum_strategy.py:320-416
    ins, outs = [], []
    terms, sid, _ = _core_terms(qctn, ins.append, outs.append)
    ins_stack, outs_stack = list(ins), list(outs)
    temap = {}
    tterms = []
    for info in target.adjacency_table:
        ci = info["core_idx"]
        t = ""
        for e in info["in_edge_list"]:
            if e["neighbor_idx"] == -1:
                s = ins_stack.pop(0)
            else:
                k = _edge_key(e["neighbor_idx"], ci, e["qubit_idx"])
                if k not in temap:
                    temap[k] = get_symbol(sid)
                    sid += 1
                s = temap[k]
            t += s
        for e in info["out_edge_list"]:
            if e["neighbor_idx"] == -1:
                s = outs_stack.pop(0)
            else:
                k = _edge_key(ci, e["neighbor_idx"], e["qubit_idx"])
                if k not in temap:
                    temap[k] = get_symbol(sid)
                    sid += 1
                s = temap[k]
            t += s
        tterms.append(t)
    eq = "".join(t + "," for t in terms) + ",".join(tterms) + "->"
    return eq, qctn.core_shapes() + target.core_shapes()


# ---- workload helpers (symmetry_breaking_quantum.py) ---------------------------------------

def incidence_to_graph(incidence: np.ndarray, core_symbols=None) -> str:
    """Valid-graph branch (for_display=False) of symmetry_breaking_quantum.py:15-63."""
    if incidence.ndim != 2:
        raise ValueError("incidence must be 2D (n_qubits x n_cores)")
    if (incidence < 0).any():
        raise ValueError("incidence entries must be >= 0")
    nq, nc = incidence.shape
    if core_symbols is None:
        core_symbols = [get_symbol(i) for i in range(nc)]
    lines = []
    for q in range(nq):
        entries = [(core_symbols[c], int(incidence[q, c])) for c in range(nc) if incidence[q, c] > 0]
        if not entries:
            raise ValueError(f"Row {q} has no cores; graph line would be invalid.")
        line = f"-{entries[0][1]}-{entries[0][0]}"
        for core, dim in entries[1:]:
            line += f"-{dim}-" + core
        line += f"-{entries[-1][1]}-"
        lines.append(line)
    return "\n".join(lines)


def build_brick_wall_IM(n_qubits, n_cells, rank=2):                  # symmetry_breaking_quantum.py:107-125
    n_cores = (n_qubits - 1) * n_cells
    IM = np.zeros((n_qubits, n_cores), dtype=int)
    for cell in range(n_cells):
        base = cell * (n_qubits - 1)
        col = 0
        for q in range(0, n_qubits - 1, 2):
            IM[q, base + col] = rank
            IM[q + 1, base + col] = rank
            col += 1
        for q in range(1, n_qubits - 1, 2):
            IM[q, base + col] = rank
            IM[q + 1, base + col] = rank
            col += 1
    return IM


# ---- split / merge at graph level (qctn.py:1217-1506) --------------------------------------

def _parse_line(line):                                                # qctn.py:1217-1250
    s = line.strip().replace("-", "")
    out, i = [], 0
    while i < len(s):
        if s[i].isdigit():
            j = i
            while j < len(s) and s[j].isdigit():
                j += 1
            out.append(("dim", int(s[i:j])))
            i = j
        else:
            out.append(("core", s[i]))
            i += 1
    return out


def _rebuild(tokens):                                                 # qctn.py:1252-1265
    return "-" + "-".join(str(v) for _, v in tokens) + "-"


def split_graph(qctn: QCTNRef, split_idx=None):                       # qctn.py:1296-1391
    if split_idx is None:
        split_idx = qctn.ncores // 2
    if split_idx <= 0 or split_idx >= qctn.ncores:
        raise ValueError(f"split_idx must be between 1 and {qctn.ncores - 1}, got {split_idx}")
    g1, g2 = set(qctn.cores[:split_idx]), set(qctn.cores[split_idx:])
    l1, l2 = [], []
    for q, line in enumerate(qctn.qubits):
        toks = _parse_line(line)
        pos = [(i, t[1]) for i, t in enumerate(toks) if t[0] == "core"]
        p1 = [(i, c) for i, c in pos if c in g1]
        p2 = [(i, c) for i, c in pos if c in g2]
        if p1 and p2:
            last1 = max(i for i, _ in p1)
            first2 = min(i for i, _ in p2)
            if last1 >= first2:
                raise ValueError(f"Cannot split: cores from both groups are interleaved on qubit {q}.")
            l1.append(_rebuild(toks[: last1 + 2]))
            l2.append(_rebuild(toks[first2 - 1:]))
        elif p1:
            l1.append(_rebuild(toks))
        elif p2:
            l2.append(_rebuild(toks))
    if not l1:
        raise ValueError("After split, Group 1 has no qubit lines.")
    if not l2:
        raise ValueError("After split, Group 2 has no qubit lines.")
    return "\n".join(l1), "\n".join(l2)


def merge_graphs(q1: QCTNRef, q2: QCTNRef):                           # qctn.py:1403-1493
    n1, n2 = q1.nqubits, q2.nqubits
    total = q1.ncores + q2.ncores
    syms = [get_symbol(i) for i in range(total)]
    m1 = {old: syms[i] for i, old in enumerate(q1.cores)}
    m2 = {old: syms[q1.ncores + i] for i, old in enumerate(q2.cores)}
    r1 = ["".join(m1.get(ch, ch) for ch in l) for l in q1.qubits]
    r2 = ["".join(m2.get(ch, ch) for ch in l) for l in q2.qubits]
    pw1 = max(len(l) for l in r1) - 3
    pw2 = max(len(l) for l in r2) - 3
    lines = []
    for qi in range(max(n1, n2)):
        h1, h2 = qi < n1, qi < n2
        a = r1[qi] if h1 else "-" * pw1
        b = r2[qi] if h2 else "-" * pw2
        ma = re.search(r"-\d+-$", a)
        da = ma.group() if h1 else ""
        sa = a[: ma.start()] if h1 else a
        mb = re.match(r"^-\d+-", b)
        db = mb.group() if h2 else ""
        sb = b[mb.end():] if h2 else b
        if h1 and h2:
            lines.append(sa + da + sb)
        elif h1:
            lines.append(sa + sb + da)
        else:
            lines.append(db + sa + sb)
    return "\n".join(lines), m1, m2


# ---- deterministic cores -------------------------------------------------------------------

def haar_unitary(rng: np.random.Generator, n: int, dtype=np.complex128) -> np.ndarray:
    """Random unitary by complex QR with phase fix (the construction of
    tneq_qc/backends/backend_pytorch.py:470-495, here driven by numpy's RNG)."""
    z = (rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))) / np.sqrt(2.0)
    q, r = np.linalg.qr(z)
    d = np.diag(r)
    q = q @ np.diag((d / np.abs(d)).conj())
    return q.astype(dtype)


def random_cores(qctn: QCTNRef, seed: int, dtype=np.complex128, kind="unitary"):
    """One tensor per core (core order), shape input_shape + output_shape (qctn.py:741-757)."""
    rng = np.random.default_rng(seed)
    out = {}
    for info in qctn.adjacency_table:
        shape = tuple(info["input_shape"] + info["output_shape"])
        din, dout = info["input_dim"], info["output_dim"]
        if kind == "identity":
            m = np.eye(din, dout)
        elif kind == "unitary" and din == dout:
            m = haar_unitary(rng, din)
        else:
            m = rng.standard_normal((din, dout)) + 1j * rng.standard_normal((din, dout))
        if not np.iscomplexobj(np.zeros(1, dtype=dtype)):
            m = m.real
        out[info["core_name"]] = np.ascontiguousarray(m.astype(dtype).reshape(shape))
    return out
