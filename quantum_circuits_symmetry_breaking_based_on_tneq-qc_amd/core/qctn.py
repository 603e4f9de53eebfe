"""QCTN host mirror: graph string -> per-core edge table -> core shapes / weights.

Same public surface and bookkeeping as tneq_qc/core/qctn.py (the reference cannot be imported
here): core order (qctn.py:497-506), the adjacency_table and core axis layout
input_shape + output_shape (qctn.py:591-760), set/save/load (qctn.py:762-983), split/merge
(qctn.py:1296-1522).  Index bookkeeping is bit-exact with the reference rules; tests check it
against the oracle restatement and hand-derived fixtures.

Parsing here is token based (each qubit line is dim, core, dim, core, ..., dim once dashes are
removed) instead of the reference's three regexes; for well-formed lines both give the same
edges in the same order: for every line in qubit order, the first core gets the circuit-input
edge, the last core the circuit-output edge, consecutive cores a connection edge.
"""
from __future__ import annotations

import re
from pathlib import Path
from typing import Any, Dict, List, Mapping, Optional, Tuple, Union

import numpy as np

from ..einsum import get_symbol
from .tn_tensor import TNTensor

_SYM_INDEX = {get_symbol(i): i for i in range(10000)}


def _tokens(line: str) -> List[Tuple[str, Any]]:
    """'-2-A-5-B-3-' -> [('dim',2),('core','A'),('dim',5),('core','B'),('dim',3)] (qctn.py:1217-1250)."""
    s = line.strip().replace("-", "")
    out: List[Tuple[str, Any]] = []
    i = 0
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


def _line_string(tokens) -> str:
    return "-" + "-".join(str(v) for _, v in tokens) + "-"


class QCTN:
    """Quantum-circuit tensor network (rows = qubit lines, symbols = cores, numbers = bond ranks)."""

    def __init__(self, graph: str, backend=None):
        self.qubits = graph.strip().splitlines()
        self.nqubits = len(self.qubits)
        self.qubit_indices = list(range(self.nqubits))
        self.graph = graph
        cores = {c for c in graph if c in _SYM_INDEX}
        self.cores = sorted(cores, key=lambda c: _SYM_INDEX[c])
        self.ncores = len(self.cores)
        self.dict_core2idx = {c: i for i, c in enumerate(self.cores)}
        self._build_adjacency()
        self.backend = backend
        self._loaded_metadata: Optional[Mapping[str, str]] = None
        self.cores_weights: Dict[str, Any] = {}
        if backend is not None:
            self._init_cores()

    # ---------------------------------------------------------------- bookkeeping
    def _build_adjacency(self):
        tab = [{"core_idx": i, "core_name": c, "in_edge_list": [], "out_edge_list": [],
                "input_shape": [], "output_shape": [], "input_dim": 1, "output_dim": 1}
               for i, c in enumerate(self.cores)]
        idx = self.dict_core2idx
        for q, line in enumerate(self.qubits):
            toks = _tokens(line)
            if len(toks) < 3 or toks[0][0] != "dim" or toks[-1][0] != "dim":
                raise ValueError(f"qubit line {q} is malformed: {line!r}")
            seq = []  # (core, rank_after)
            for k in range(1, len(toks) - 1, 2):
                if toks[k][0] != "core" or toks[k + 1][0] != "dim":
                    raise ValueError(f"qubit line {q} is malformed: {line!r}")
                seq.append((toks[k][1], toks[k + 1][1]))
            first, last = seq[0][0], seq[-1][0]
            tab[idx[first]]["in_edge_list"].append(
                {"neighbor_idx": -1, "neighbor_name": "", "edge_rank": toks[0][1], "qubit_idx": q})
            tab[idx[last]]["out_edge_list"].append(
                {"neighbor_idx": -1, "neighbor_name": "", "edge_rank": toks[-1][1], "qubit_idx": q})
            for (c1, r1), (c2, _) in zip(seq[:-1], seq[1:]):
                tab[idx[c1]]["out_edge_list"].append(
                    {"neighbor_idx": idx[c2], "neighbor_name": c2, "edge_rank": r1, "qubit_idx": q})
                tab[idx[c2]]["in_edge_list"].append(
                    {"neighbor_idx": idx[c1], "neighbor_name": c1, "edge_rank": r1, "qubit_idx": q})
        for t in tab:
            t["input_shape"] = [e["edge_rank"] for e in t["in_edge_list"]]
            t["output_shape"] = [e["edge_rank"] for e in t["out_edge_list"]]
            t["input_dim"] = int(np.prod(t["input_shape"])) if t["input_shape"] else 1
            t["output_dim"] = int(np.prod(t["output_shape"])) if t["output_shape"] else 1
        self.adjacency_table = tab
        n = self.ncores
        adj = np.empty((n, n), dtype=object)
        for i in range(n):
            for j in range(n):
                adj[i, j] = []
        for t in tab:
            for e in t["out_edge_list"]:
                if e["neighbor_idx"] >= 0:
                    adj[t["core_idx"], e["neighbor_idx"]].append(e["edge_rank"])
                    adj[e["neighbor_idx"], t["core_idx"]].append(e["edge_rank"])
        self.adjacency_matrix = adj
        ins = np.empty(n, dtype=object)
        outs = np.empty(n, dtype=object)
        for i in range(n):
            ins[i] = list(tab[i]["input_shape"])
            outs[i] = list(tab[i]["output_shape"])
        self.circuit = (ins, adj, outs)

    def core_shape(self, name: str) -> Tuple[int, ...]:
        t = self.adjacency_table[self.dict_core2idx[name]]
        return tuple(t["input_shape"] + t["output_shape"])

    def core_qubits(self, name: str) -> List[int]:
        t = self.adjacency_table[self.dict_core2idx[name]]
        return sorted({e["qubit_idx"] for e in t["in_edge_list"]})

    # ---------------------------------------------------------------- weights
    def _init_cores(self):
        """qctn.py:724-760: init_random_core([in_dim, out_dim]) reshaped to in_shape + out_shape."""
        for t in self.adjacency_table:
            core = self.backend.init_random_core([t["input_dim"], t["output_dim"]])
            raw = core.tensor if isinstance(core, TNTensor) else core
            raw = raw.reshape(t["input_shape"] + t["output_shape"])
            self.cores_weights[t["core_name"]] = TNTensor(raw, core.scale) if isinstance(core, TNTensor) else raw

    def set_cores(self, cores, strict: bool = True):
        """qctn.py:762-900 (list by position / dict by name, numel-checked, reshaped)."""
        import warnings
        if isinstance(cores, list):
            if strict and len(cores) != self.ncores:
                raise ValueError(f"strict=True: expected {self.ncores} core tensors, got {len(cores)}.")
            n = min(len(cores), self.ncores)
            if not strict and len(cores) != self.ncores:
                warnings.warn(f"strict=False: input list has {len(cores)} tensors but QCTN has "
                              f"{self.ncores} cores. Only the first {n} will be set.", stacklevel=2)
            for i in range(n):
                self._set_single_core(self.cores[i], cores[i])
        elif isinstance(cores, dict):
            keys, mine = set(cores), set(self.cores)
            if strict and keys != mine:
                parts = []
                if mine - keys:
                    parts.append(f"missing keys ({len(mine - keys)}): {mine - keys}")
                if keys - mine:
                    parts.append(f"extra keys ({len(keys - mine)}): {keys - mine}")
                raise ValueError(f"strict=True: key mismatch — {'; '.join(parts)}.")
            for name in self.cores:
                if name in cores:
                    self._set_single_core(name, cores[name])
        else:
            raise TypeError(f"cores must be a list or dict, got {type(cores).__name__}")

    def _set_single_core(self, name: str, tensor):
        target = self.core_shape(name)
        src = tuple(tensor.shape)
        if int(np.prod(src)) != int(np.prod(target)):
            raise ValueError(f"Core '{name}': size mismatch — input has {int(np.prod(src))} elements "
                             f"(shape {src}) but target has {int(np.prod(target))} elements (shape {target}).")
        if src != target:
            tensor = tensor.reshape(list(target))
        self.cores_weights[name] = tensor

    def save_cores(self, file_path: Union[str, Path], metadata: Optional[Mapping[str, str]] = None):
        """safetensors, keys core_{name} or core_{name}_real/_imag (qctn.py:902-926)."""
        if self.backend is None:
            raise RuntimeError("Backend must be initialized before saving cores.")
        from safetensors.numpy import save_file
        d = {}
        for name, t in self.cores_weights.items():
            arr = self.backend.tensor_to_numpy(t.tensor * t.scale if isinstance(t, TNTensor) else t)
            if np.iscomplexobj(arr):
                d[f"core_{name}_real"] = np.ascontiguousarray(arr.real)
                d[f"core_{name}_imag"] = np.ascontiguousarray(arr.imag)
            else:
                d[f"core_{name}"] = np.ascontiguousarray(arr)
        save_file(d, str(file_path), metadata={str(k): str(v) for k, v in (metadata or {}).items()})

    def load_cores(self, file_path: Union[str, Path], strict: bool = True) -> Mapping[str, str]:
        """qctn.py:928-964: loaded cores become auto-scaled TNTensors (tensor / max|tensor|, scale =
        max|tensor|).  Returns the metadata the reference returns: its `load_file` result is a plain
        dict (never a (tensors, metadata) tuple, qctn.py:944-949), so that is always {}."""
        if self.backend is None:
            raise RuntimeError("Backend must be initialized before loading cores.")
        from safetensors.numpy import load_file
        d = load_file(str(file_path))
        meta = {}
        for name in self.cores:
            k, kr, ki = f"core_{name}", f"core_{name}_real", f"core_{name}_imag"
            if kr in d:
                arr = d[kr] + 1j * d[ki]
            elif k in d:
                arr = d[k]
            else:
                if strict:
                    raise KeyError(f"Missing tensor for core {name} in {file_path}")
                continue
            tn = TNTensor(self.backend.convert_to_tensor(arr))
            tn.auto_scale()
            self.cores_weights[name] = tn
        self._loaded_metadata = {str(k): str(v) for k, v in meta.items()}
        return self._loaded_metadata

    @classmethod
    def from_pretrained(cls, graph: str, file_path, backend=None, strict: bool = True) -> "QCTN":
        if backend is None:
            from ..backends.backend_factory import BackendFactory
            backend = BackendFactory.get_default_backend()
        inst = cls(graph, backend=backend)
        inst.load_cores(file_path, strict=strict)
        return inst

    # ---------------------------------------------------------------- split / merge
    def split(self, split_idx: Optional[int] = None) -> Tuple["QCTN", "QCTN"]:
        """qctn.py:1296-1401: group 1 = cores[:split_idx], group 2 = the rest; the boundary rank
        becomes group 1's output rank and group 2's input rank on every shared line."""
        if split_idx is None:
            split_idx = self.ncores // 2
        if split_idx <= 0 or split_idx >= self.ncores:
            raise ValueError(f"split_idx must be between 1 and {self.ncores - 1}, got {split_idx}")
        g1, g2 = set(self.cores[:split_idx]), set(self.cores[split_idx:])
        l1, l2 = [], []
        for q, line in enumerate(self.qubits):
            toks = _tokens(line)
            pos = [(i, v) for i, (k, v) in enumerate(toks) if k == "core"]
            p1 = [i for i, c in pos if c in g1]
            p2 = [i for i, c in pos if c in g2]
            if p1 and p2:
                if max(p1) >= min(p2):
                    raise ValueError(f"Cannot split: cores from both groups are interleaved on qubit {q}. "
                                     f"Ensure that all Group-1 cores appear before Group-2 cores on every qubit line.")
                l1.append(_line_string(toks[: max(p1) + 2]))
                l2.append(_line_string(toks[min(p2) - 1:]))
            elif p1:
                l1.append(_line_string(toks))
            elif p2:
                l2.append(_line_string(toks))
        if not l1:
            raise ValueError("After split, Group 1 has no qubit lines. All qubits belong to Group 2.")
        if not l2:
            raise ValueError("After split, Group 2 has no qubit lines. All qubits belong to Group 1.")
        q1 = QCTN("\n".join(l1), backend=None)
        q2 = QCTN("\n".join(l2), backend=None)
        q1.backend = q2.backend = self.backend
        for name in self.cores[:split_idx]:
            if name in self.cores_weights:
                q1.cores_weights[name] = self.cores_weights[name]
        for name in self.cores[split_idx:]:
            if name in self.cores_weights:
                q2.cores_weights[name] = self.cores_weights[name]
        return q1, q2

    @staticmethod
    def merge(qctn1: "QCTN", qctn2: "QCTN") -> "QCTN":
        """qctn.py:1403-1506: horizontal concatenation, shared boundary kept once, cores renamed
        get_symbol(0..) in order (qctn1's first), shorter side padded with dashes at the bottom."""
        n1, n2 = qctn1.nqubits, qctn2.nqubits
        syms = [get_symbol(i) for i in range(qctn1.ncores + qctn2.ncores)]
        m1 = {old: syms[i] for i, old in enumerate(qctn1.cores)}
        m2 = {old: syms[qctn1.ncores + i] for i, old in enumerate(qctn2.cores)}
        r1 = ["".join(m1.get(ch, ch) for ch in l) for l in qctn1.qubits]
        r2 = ["".join(m2.get(ch, ch) for ch in l) for l in qctn2.qubits]
        pad1 = max(len(l) for l in r1) - 3
        pad2 = max(len(l) for l in r2) - 3
        lines = []
        for qi in range(max(n1, n2)):
            h1, h2 = qi < n1, qi < n2
            a = r1[qi] if h1 else "-" * pad1
            b = r2[qi] if h2 else "-" * pad2
            if h1:
                ma = re.search(r"-\d+-$", a)
                da, sa = ma.group(), a[: ma.start()]
            else:
                da, sa = "", a
            if h2:
                mb = re.match(r"^-\d+-", b)
                db, sb = mb.group(), b[mb.end():]
            else:
                db, sb = "", b
            if h1 and h2:
                lines.append(sa + da + sb)
            elif h1:
                lines.append(sa + sb + da)
            else:
                lines.append(db + sa + sb)
        backend = qctn1.backend if qctn1.backend is not None else qctn2.backend
        new = QCTN("\n".join(lines), backend=None)
        new.backend = backend
        for old, nw in m1.items():
            if old in qctn1.cores_weights:
                new.cores_weights[nw] = qctn1.cores_weights[old]
        for old, nw in m2.items():
            if old in qctn2.cores_weights:
                new.cores_weights[nw] = qctn2.cores_weights[old]
        return new

    def merge_with(self, other: "QCTN") -> "QCTN":
        return QCTN.merge(self, other)

    def __repr__(self):
        return f"QCTN(nqubits={self.nqubits}, ncores={self.ncores})"
