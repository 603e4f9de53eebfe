"""EinsumStrategy: einsum-equation builders + HIP contraction expressions.

Mirror of tneq_qc/contractor/einsum_strategy.py.  The equation strings are bit-identical to the
reference's (same symbol numbering: one get_symbol per circuit input/output and per internal edge
keyed by (sorted core pair, qubit), walked core by core, in-edges then out-edges — lines 136-194),
so output axes come out in the reference's core order.  ``create_contract_expression`` returns a
HipContractExpression instead of an opt_einsum ContractExpression (same call protocol).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

from ..core.tn_tensor import TNTensor
from ..einsum import get_symbol
from ..expression import HipContractExpression
from .base import ContractionStrategy


@dataclass
class _Walk:
    """Result of one pass over the adjacency table (einsum_strategy.py:155-187)."""
    terms: List[str]                                   # one term per core, core order
    inputs: List[Tuple[str, int]] = field(default_factory=list)   # (symbol, qubit) in core order
    outputs: List[Tuple[str, int]] = field(default_factory=list)  # (symbol, qubit) in core order
    circuit: List[str] = field(default_factory=list)              # all circuit legs, creation order
    next_id: int = 0
    edges: Dict[tuple, str] = field(default_factory=dict)


def walk_cores(qctn, start_id: int = 0) -> _Walk:
    w = _Walk(terms=[], next_id=start_id)

    def fresh() -> str:
        s = get_symbol(w.next_id)
        w.next_id += 1
        return s

    for info in qctn.adjacency_table:
        me = info["core_idx"]
        term = []
        for kind, edges in (("in", info["in_edge_list"]), ("out", info["out_edge_list"])):
            for e in edges:
                nb = e["neighbor_idx"]
                if nb == -1:
                    s = fresh()
                    (w.inputs if kind == "in" else w.outputs).append((s, e["qubit_idx"]))
                    w.circuit.append(s)
                else:
                    key = (min(nb, me), max(nb, me), e["qubit_idx"])
                    s = w.edges.get(key)
                    if s is None:
                        s = w.edges[key] = fresh()
                term.append(s)
        w.terms.append("".join(term))
    return w


def _core_shapes(qctn):
    return [tuple(qctn.cores_weights[c].shape) if c in qctn.cores_weights else qctn.core_shape(c)
            for c in qctn.cores]


class EinsumStrategy(ContractionStrategy):
    """'fast' mode strategy: one einsum for the whole network, run by a HIP expression."""

    def check_compatibility(self, qctn, shapes_info: Dict[str, Any]) -> bool:
        return True

    def get_compute_function(self, qctn, shapes_info: Dict[str, Any], backend, **kw) -> Callable:
        """einsum_strategy.py:24-110: build_with_self_expression, then states + cores + Mx +
        reversed cores + states (cores NOT conjugated on the right, as in the reference)."""
        eq, shapes = self.build_with_self_expression(
            qctn, shapes_info.get("circuit_states_shapes"), shapes_info.get("measure_shapes"),
            shapes_info.get("measure_is_matrix", True))
        expr = self.create_contract_expression(eq, shapes)

        def compute_fn(cores_dict, circuit_states, measure_matrices, right_cores_dict=None):
            tensors = []
            if circuit_states is not None:
                tensors.extend(circuit_states if isinstance(circuit_states, list) else [circuit_states])
            tensors.extend(cores_dict[c] for c in qctn.cores)
            if measure_matrices is not None:
                tensors.extend(measure_matrices if isinstance(measure_matrices, list) else [measure_matrices])
            tensors.extend(cores_dict[c] for c in reversed(qctn.cores))
            if circuit_states is not None:
                tensors.extend(circuit_states if isinstance(circuit_states, list) else [circuit_states])
            raw, scale = [], None
            for t in tensors:
                if isinstance(t, TNTensor):
                    raw.append(t.tensor)
                    scale = t.scale if scale is None else scale * t.scale
                else:
                    raw.append(t)
            res = backend.execute_expression(backend.jit_compile(expr), *raw)
            return TNTensor(res, scale=scale) if scale is not None else res

        return compute_fn

    def estimate_cost(self, qctn, shapes_info: Dict[str, Any]) -> float:
        return 1.0  # einsum_strategy.py:130

    @property
    def name(self) -> str:
        return "einsum_default"

    # ------------------------------------------------------------------ builders
    @staticmethod
    def build_core_only_expression(qctn) -> Tuple[str, List]:
        """einsum_strategy.py:136-194 — output = every core's circuit in/out legs, core order."""
        w = walk_cores(qctn)
        rhs = "".join(w.circuit)
        return ",".join(w.terms) + "->" + rhs, _core_shapes(qctn)

    @staticmethod
    def build_with_inputs_expression(qctn, inputs_shape) -> Tuple[str, List]:
        """einsum_strategy.py:196-256 — one input tensor carrying all circuit-input legs."""
        w = walk_cores(qctn)
        lhs = "".join(s for s, _ in w.inputs) + "," + ",".join(w.terms)
        return lhs + "->" + "".join(s for s, _ in w.outputs), [tuple(inputs_shape)] + _core_shapes(qctn)

    @staticmethod
    def build_with_vector_inputs_expression(qctn, inputs_shapes: List) -> Tuple[str, List]:
        """einsum_strategy.py:258-318 — one vector per circuit input, consumed in core/in-edge
        order; open outputs in core order."""
        w = walk_cores(qctn)
        lhs = "".join(s + "," for s, _ in w.inputs) + ",".join(w.terms)
        return lhs + "->" + "".join(s for s, _ in w.outputs), \
            [tuple(s) for s in inputs_shapes] + _core_shapes(qctn)

    @staticmethod
    def build_with_qctn_expression(qctn, target_qctn) -> Tuple[str, List]:
        """einsum_strategy.py:320-416 — target's circuit inputs reuse qctn's input symbols and its
        outputs qctn's output symbols (stack order), full contraction to a scalar."""
        w = walk_cores(qctn)
        ins = [s for s, _ in w.inputs]
        outs = [s for s, _ in w.outputs]
        nid = w.next_id
        tmap: Dict[tuple, str] = {}
        terms = []
        for info in target_qctn.adjacency_table:
            me = info["core_idx"]
            t = ""
            for kind, edges in (("in", info["in_edge_list"]), ("out", info["out_edge_list"])):
                for e in edges:
                    nb = e["neighbor_idx"]
                    if nb == -1:
                        t += (ins if kind == "in" else outs).pop(0)
                    else:
                        key = (min(nb, me), max(nb, me), e["qubit_idx"])
                        if key not in tmap:
                            tmap[key] = get_symbol(nid)
                            nid += 1
                        t += tmap[key]
            terms.append(t)
        eq = "".join(t + "," for t in w.terms) + ",".join(terms) + "->"
        return eq, _core_shapes(qctn) + _core_shapes(target_qctn)

    @staticmethod
    def build_with_self_expression(qctn, circuit_states_shape=None, measure_shape=None,
                                   measure_is_matrix=False) -> Tuple[str, List]:
        """einsum_strategy.py:418-620, including its quirk of swapping the last two measurement
        blocks (lines 517-519)."""
        is_states_list = (isinstance(circuit_states_shape, tuple) and bool(circuit_states_shape)
                          and isinstance(circuit_states_shape[0], tuple))
        is_measure_list = (isinstance(measure_shape, tuple) and bool(measure_shape)
                           and isinstance(measure_shape[0], tuple))
        w = walk_cores(qctn)
        sid = w.next_id
        ins = [s for s, _ in w.inputs]
        outs = [s for s, _ in w.outputs]
        mid_map = {c: c for c in outs}
        batch = ""
        middle: List[str] = []
        if measure_shape is not None:
            batch = get_symbol(sid)
            sid += 1
            for c in outs:
                s = get_symbol(sid)
                sid += 1
                mid_map[c] = s
                middle.append(batch + c + s)
            if len(middle) >= 2:
                middle = middle[:-2] + middle[-2:][::-1]
        new_map: Dict[str, str] = {}
        inv_terms = []
        outset = set(outs)
        for term in reversed(w.terms):
            t = ""
            for ch in term:
                if ch in outset:
                    t += mid_map[ch]
                else:
                    if ch not in new_map:
                        new_map[ch] = get_symbol(sid)
                        sid += 1
                    t += new_map[ch]
            inv_terms.append(t)
        body = ",".join(w.terms + middle + inv_terms)
        if is_states_list:
            left_states = ",".join(ins)
            right_states = ",".join(new_map[c] for c in reversed(ins))
        else:
            left_states = "".join(ins)
            right_states = "".join(new_map[c] for c in reversed(ins))
        parts = []
        if circuit_states_shape is not None:
            parts.append(left_states)
        parts.append(body)
        if circuit_states_shape is not None:
            parts.append(right_states)
        eq = ",".join(parts) + "->" + batch
        shapes: List = []
        if circuit_states_shape is not None:
            shapes.extend(list(circuit_states_shape) if is_states_list else [circuit_states_shape])
        shapes.extend(_core_shapes(qctn))
        if measure_shape is not None:
            shapes.extend(list(measure_shape) if is_measure_list else [measure_shape])
        shapes.extend(_core_shapes(qctn)[::-1])
        if circuit_states_shape is not None:
            shapes.extend(list(circuit_states_shape) if is_states_list else [circuit_states_shape])
        return eq, shapes

    @staticmethod
    def build_amplitude_expression(qctn, fixed_outputs: Dict[int, int], input_dim: int = 2,
                                   output_dim: int = 2):
        """Extension for amplitude batches: the vector-inputs network of
        build_with_vector_inputs_expression plus one projector vector <x_q| per fixed output qubit.
        Operand order: input vectors (core order), cores, then the projectors (core order of the
        outputs); the open outputs stay in core order.  Returns (eq, shapes, fixed_qubits_order,
        open_qubits_order)."""
        w = walk_cores(qctn)
        proj = [(s, q) for s, q in w.outputs if q in fixed_outputs]
        open_ = [(s, q) for s, q in w.outputs if q not in fixed_outputs]
        lhs = "".join(s + "," for s, _ in w.inputs) + ",".join(w.terms)
        lhs += "".join("," + s for s, _ in proj)
        shapes = [(input_dim,)] * len(w.inputs) + _core_shapes(qctn) + [(output_dim,)] * len(proj)
        return (lhs + "->" + "".join(s for s, _ in open_), shapes,
                [q for _, q in w.inputs], [q for _, q in proj], [q for _, q in open_])

    @staticmethod
    def create_contract_expression(einsum_equation: str, tensor_shapes: List, optimize="auto",
                                   **kw) -> HipContractExpression:
        """einsum_strategy.py:622-643; 'auto' resolves to Configuration.opt_einsum_optimize =
        'greedy' in the reference (config.py:3), same here."""
        opt = optimize if optimize != "auto" else "greedy"
        return HipContractExpression(einsum_equation, *tensor_shapes, optimize=opt, **kw)
