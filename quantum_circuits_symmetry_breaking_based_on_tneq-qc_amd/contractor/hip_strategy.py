"""HipTreeStrategy — the 'balanced'/'full' executor on the MI355X.

Computes exactly what GreedyStrategy.get_compute_function's compute_fn computes
(tneq_qc/contractor/greedy_strategy.py:41-1080) — the L·M·R network
    result[batch] = sum  states_L · cores_L · Mx · cores_R · states_R
(L = the cores, M = one Mx per qubit with batch symbols 'a' / 'ab', R = conj(core) for
right_qctn="symmetric" or a right QCTN's cores) including the reference's bookkeeping
behaviour for open legs and right QCTNs: the reference's qubit-group sweep is replayed on axis
labels (contractor/greedy_symbolic.py) and folded into ONE einsum over the leaf operands, which
runs as one native plan (HipContractExpression: path found once per shape key, tree on the GPU)
instead of one torch.einsum per group.  TNTensor scales multiply on the host (:912-957).
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Tuple

from ..core.tn_tensor import TNTensor
from ..expression import HipContractExpression
from .base import ContractionStrategy
from .greedy_symbolic import greedy_equation


def _present(container, q) -> bool:
    """greedy_strategy.py:82-99, :141-156: dict -> key present, list/tuple -> index in range."""
    if container is None:
        return False
    if isinstance(container, dict):
        return q in container
    if isinstance(container, (list, tuple)):
        return q < len(container)
    raise TypeError(f"unsupported container type {type(container).__name__}")


class HipTreeStrategy(ContractionStrategy):
    """L·M·R contraction on the HIP tree executor (registered for 'balanced' and 'full')."""

    def check_compatibility(self, qctn, shapes_info: Dict[str, Any]) -> bool:
        """Always True, as GreedyStrategy (greedy_strategy.py:35-39): the replay covers closed
        sandwiches, open legs and right QCTNs alike."""
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
            qs = qctn.qubit_indices
            states = {q: circuit_states[q] for q in qs if _present(circuit_states, q)}
            mx = {q: measure_matrices[q] for q in qs
                  if _present(measure_matrices, q) and measure_matrices[q] is not None}
            cores = {c: cores_dict[c] for c in qctn.cores}
            rcores = None
            if right_qctn is not None and not isinstance(right_qctn, str):
                if right_cores_dict is None:
                    raise ValueError("right_qctn given without right_cores_dict")
                rcores = {c: right_cores_dict[c] for c in right_qctn.cores}
            key = (tuple((q, tuple(s.shape)) for q, s in states.items()),
                   tuple((q, tuple(m.shape)) for q, m in mx.items()),
                   tuple(tuple(t.shape) for t in cores.values()),
                   tuple(tuple(t.shape) for t in rcores.values()) if rcores else None)
            hit = cache.get(key)
            if hit is None:
                eq, recipe = greedy_equation(
                    qctn, {q: s.shape[0] for q, s in states.items()},
                    {q: (m.ndim, m.shape[-2], m.shape[-1]) for q, m in mx.items()},
                    {c: len(t.shape) for c, t in cores.items()}, right_qctn,
                    {c: len(t.shape) for c, t in rcores.items()} if rcores else None)
                shapes = [tuple(_operand(r, cores, rcores, states, mx).shape) for r in recipe]
                hit = (HipContractExpression(eq, *shapes, optimize="greedy"), recipe)
                cache[key] = hit
            expr, recipe = hit
            raw, scale, log_scale = [], None, None
            for r in recipe:
                t = _operand(r, cores, rcores, states, mx)
                if isinstance(t, TNTensor):
                    # every use multiplies its scale in (a core twice: its L and its R copy)
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


def _operand(r, cores, rcores, states, mx):
    kind, key = r
    if kind in ("L", "R"):
        return cores[key]
    if kind == "Rq":
        return rcores[key]
    if kind == "S":
        return states[key]
    return mx[key]
