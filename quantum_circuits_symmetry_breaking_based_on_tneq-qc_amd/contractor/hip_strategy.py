"""HipTreeStrategy — the 'balanced'/'full' executor on the MI355X.

Computes exactly what GreedyStrategy.get_compute_function's compute_fn computes
(tneq_qc/contractor/greedy_strategy.py:41-600): the symmetric L·M·R network
    result[batch] = sum  states_L · cores_L · Mx · cores_R · states_R
with
  * L = the cores as given, circuit states attached to their circuit-input legs (:105-138),
  * M = one Mx per qubit, batch symbols 'a' (3-D Mx) or 'ab' (4-D Mx) shared by all Mx,
        Mx dim -2 on the L circuit-output leg, dim -1 on the R side (:140-190, :329-373),
  * R (right_qctn="symmetric") = conj(core) for complex cores (`_get_tensor` :675-681) with the
        same axis meaning, the circuit states attached to its circuit-input legs (:192-223, :262-295);
    R (right_qctn=QCTN) = the right QCTN's cores NOT conjugated, their circuit inputs facing Mx and
        outputs facing the states, each right core's axes read in fully reversed order — the effect
        of the dim map at :764-822 with `original_in_edge_count` never set,
  * TNTensor scales multiplied on the host (:912-957).
Instead of the reference's Python qubit sweep with one torch.einsum per group, the whole
network is one HipContractExpression: the path is found once, the tree runs as one native plan.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Tuple

from ..core.tn_tensor import TNTensor
from ..einsum import get_symbol
from ..expression import HipContractExpression
from .base import ContractionStrategy


def _per_qubit(container, q):
    """Entry for qubit q from a list/tuple/dict container (greedy_strategy.py:108-118, 143-158)."""
    if container is None:
        return None
    if isinstance(container, dict):
        return container.get(q)
    if isinstance(container, (list, tuple)):
        return container[q] if q < len(container) else None
    raise TypeError(f"unsupported container type {type(container).__name__}")


class _Symbols:
    def __init__(self):
        self.i = 2  # 'a', 'b' reserved for batch (greedy_strategy.py:411-417)

    def __call__(self) -> str:
        s = get_symbol(self.i)
        self.i += 1
        return s


def build_sandwich(qctn, states_dims: Dict[int, int], mx_ndims: Dict[int, int],
                   right_qctn="symmetric"):
    """Equation + operand recipe of the L·M·R network.

    Returns (equation, recipe) where recipe lists operands as tuples
    ('L', core) | ('R', core) | ('Rq', core of right_qctn) | ('SL', q) | ('SR', q) | ('M', q)."""
    sym = _Symbols()
    n = qctn.nqubits
    for q in range(n):
        if q not in mx_ndims:
            raise NotImplementedError(f"HIP sandwich needs a measurement matrix on every qubit (missing {q})")
    # ---- left cores
    lmap: Dict[tuple, str] = {}
    lin: Dict[int, str] = {}
    lout: Dict[int, str] = {}
    terms: List[str] = []
    recipe: List[tuple] = []
    for info in qctn.adjacency_table:
        me = info["core_idx"]
        t = ""
        for kind, edges in (("in", info["in_edge_list"]), ("out", info["out_edge_list"])):
            for e in edges:
                q = e["qubit_idx"]
                if e["neighbor_idx"] == -1:
                    d = lin if kind == "in" else lout
                    d[q] = sym()
                    t += d[q]
                else:
                    k = (min(me, e["neighbor_idx"]), max(me, e["neighbor_idx"]), q)
                    if k not in lmap:
                        lmap[k] = sym()
                    t += lmap[k]
        terms.append(t)
        recipe.append(("L", info["core_name"]))
    # ---- right side
    rmap: Dict[tuple, str] = {}
    r_meas: Dict[int, str] = {}   # R leg facing Mx on qubit q
    r_state: Dict[int, str] = {}  # R leg facing the circuit state on qubit q
    if isinstance(right_qctn, str) and right_qctn == "symmetric":
        for info in qctn.adjacency_table:
            me = info["core_idx"]
            t = ""
            for kind, edges in (("in", info["in_edge_list"]), ("out", info["out_edge_list"])):
                for e in edges:
                    q = e["qubit_idx"]
                    if e["neighbor_idx"] == -1:
                        d = r_state if kind == "in" else r_meas
                        d[q] = sym()
                        t += d[q]
                    else:
                        k = (min(me, e["neighbor_idx"]), max(me, e["neighbor_idx"]), q)
                        if k not in rmap:
                            rmap[k] = sym()
                        t += rmap[k]
            terms.append(t)
            recipe.append(("R", info["core_name"]))
    elif right_qctn is not None and hasattr(right_qctn, "adjacency_table"):
        for info in right_qctn.adjacency_table:
            me = info["core_idx"]
            legs = []
            for kind, edges in (("in", info["in_edge_list"]), ("out", info["out_edge_list"])):
                for e in edges:
                    q = e["qubit_idx"]
                    if e["neighbor_idx"] == -1:
                        d = r_meas if kind == "in" else r_state
                        d[q] = sym()
                        legs.append(d[q])
                    else:
                        k = (min(me, e["neighbor_idx"]), max(me, e["neighbor_idx"]), q)
                        if k not in rmap:
                            rmap[k] = sym()
                        legs.append(rmap[k])
            terms.append("".join(reversed(legs)))
            recipe.append(("Rq", info["core_name"]))
    elif right_qctn is None:
        pass
    else:
        raise ValueError("Invalid right_qctn parameter.")
    # ---- measurements and states
    has_b = False
    for q in range(n):
        nd = mx_ndims[q]
        batch = "a" if nd == 3 else ("ab" if nd == 4 else "")
        has_b |= nd == 4
        if q not in lout or q not in r_meas:
            raise NotImplementedError(f"qubit {q} has no circuit output on both sides")
        terms.append(batch + lout[q] + r_meas[q])
        recipe.append(("M", q))
    for q in range(n):
        if q in lin:
            if q not in states_dims:
                raise NotImplementedError(f"HIP sandwich needs a circuit state on every input (missing {q})")
            terms.append(lin[q])
            recipe.append(("SL", q))
    for q in range(n):
        if q in r_state:
            if q not in states_dims:
                raise NotImplementedError(f"HIP sandwich needs a circuit state on every input (missing {q})")
            terms.append(r_state[q])
            recipe.append(("SR", q))
    has_a = any(v in (3, 4) for v in mx_ndims.values())
    out = ("a" if has_a else "") + ("b" if has_b else "")
    return ",".join(terms) + "->" + out, recipe


class HipTreeStrategy(ContractionStrategy):
    """L·M·R contraction on the HIP tree executor (registered for 'balanced' and 'full')."""

    def check_compatibility(self, qctn, shapes_info: Dict[str, Any]) -> bool:
        return True

    def estimate_cost(self, qctn, shapes_info: Dict[str, Any]) -> float:
        return 1e5  # below GreedyStrategy's fixed 5e5 (greedy_strategy.py:602-608) -> preferred

    @property
    def name(self) -> str:
        return "hip_tree"

    def get_compute_function(self, qctn, shapes_info: Dict[str, Any], backend,
                             right_qctn="symmetric") -> Callable:
        cache: Dict[tuple, Tuple[HipContractExpression, list]] = {}

        def compute_fn(cores_dict, circuit_states, measure_matrices, right_cores_dict=None):
            states = {q: _per_qubit(circuit_states, q) for q in range(qctn.nqubits)}
            states = {q: s for q, s in states.items() if s is not None}
            mx = {q: _per_qubit(measure_matrices, q) for q in range(qctn.nqubits)}
            mx = {q: m for q, m in mx.items() if m is not None}
            key = (tuple(sorted((q, tuple(s.shape)) for q, s in states.items())),
                   tuple(sorted((q, tuple(m.shape)) for q, m in mx.items())))
            hit = cache.get(key)
            if hit is None:
                eq, recipe = build_sandwich(qctn, {q: s.shape[0] for q, s in states.items()},
                                            {q: m.ndim for q, m in mx.items()}, right_qctn)
                shapes = [_operand(r, cores_dict, right_cores_dict, states, mx, shape_only=True)
                          for r in recipe]
                hit = (HipContractExpression(eq, *shapes, optimize="greedy"), recipe)
                cache[key] = hit
            expr, recipe = hit
            raw, scale, log_scale = [], None, None
            for r in recipe:
                t = _operand(r, cores_dict, right_cores_dict, states, mx)
                if isinstance(t, TNTensor):
                    scale = t.scale if scale is None else scale * t.scale
                    log_scale = t.log_scale if log_scale is None else log_scale + t.log_scale
                    t = t.tensor
                    if r[0] == "R" and t.is_complex():
                        t = t.conj_physical()
                raw.append(t)
            res = backend.execute_expression(expr, *raw)
            if scale is not None:
                return TNTensor(res, scale=scale, log_scale=log_scale)
            return res

        return compute_fn


def _operand(r, cores, right_cores, states, mx, shape_only=False):
    kind, key = r
    if kind == "L":
        t = cores[key]
    elif kind == "R":
        t = cores[key]
        if not shape_only and not isinstance(t, TNTensor) and t.is_complex():
            t = t.conj_physical()
    elif kind == "Rq":
        if right_cores is None:
            raise ValueError("right_qctn given without right_cores_dict")
        t = right_cores[key]
    elif kind in ("SL", "SR"):
        t = states[key]
    else:
        t = mx[key]
    return tuple(t.shape) if shape_only else t
