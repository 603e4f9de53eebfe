"""EngineSiamese caller surface (mirror of tneq_qc/core/engine_siamese.py:20-734) on the HIP backend.

contract_with_compiled_strategy keeps the reference's contract: shapes_info -> per-QCTN cached
compute_fn from the StrategyCompiler (engine_siamese.py:261-317), execute, then the Born rule
(abs_square) for complex results and TNTensor.scale_to(1.0) (engine_siamese.py:319-349).
The probability helpers follow engine_siamese.py:561-734; unlike the reference they also accept
plain-tensor results (the reference calls .scale_to on a raw tensor there).
"""
from __future__ import annotations

from typing import Any, List, Optional, Union

from ..backends.backend_factory import BackendFactory
from ..backends.backend_interface import ComputeBackend
from ..contractor import EinsumStrategy, StrategyCompiler
from .tn_tensor import TNTensor


def _shape_tuple(container):
    if container is None:
        return None
    if isinstance(container, dict):
        return tuple(container[i].shape if container[i] is not None else () for i in sorted(container))
    return tuple(s.shape if s is not None else () for s in container)


class EngineSiamese:
    def __init__(self, backend: Optional[Union[str, ComputeBackend]] = None, strategy_mode: str = "balanced"):
        if backend is None:
            self.backend = BackendFactory.get_default_backend()
        elif isinstance(backend, str):
            self.backend = BackendFactory.create_backend(backend)
        else:
            self.backend = backend
        self.contractor = EinsumStrategy()
        self.strategy_compiler = StrategyCompiler(mode=strategy_mode)
        self.strategy_mode = strategy_mode

    def contract_with_compiled_strategy(self, qctn, circuit_states_list, measure_input_list,
                                        measure_is_matrix=True, right_qctn="symmetric", ret_type="tensor"):
        states_shape = _shape_tuple(circuit_states_list)
        measure_shape = _shape_tuple(measure_input_list)
        shapes_info = {"circuit_states_shapes": states_shape, "measure_shapes": measure_shape,
                       "measure_is_matrix": measure_is_matrix}
        key = f"_compiled_strategy_{self.strategy_mode}_{states_shape}_{measure_shape}_{measure_is_matrix}"
        cached = getattr(qctn, key, None)
        if cached is None:
            fn, name, cost = self.strategy_compiler.compile(qctn, shapes_info, self.backend, right_qctn=right_qctn)
            cached = {"compute_fn": fn, "strategy_name": name, "cost": cost}
            setattr(qctn, key, cached)
        cores = {n: qctn.cores_weights[n] for n in qctn.cores}
        right_cores = None
        if right_qctn is not None and not isinstance(right_qctn, str):
            right_cores = {n: right_qctn.cores_weights[n] for n in right_qctn.cores}
        res = cached["compute_fn"](cores, circuit_states_list, measure_input_list, right_cores_dict=right_cores)
        if isinstance(res, TNTensor):
            if ret_type == "TNTensor":
                if self.backend.is_complex(res.tensor):
                    res = TNTensor(self.backend.abs_square(res.tensor), res.scale, res.log_scale)
                return res
            res.scale_to(1.0)
            return self.backend.abs_square(res.tensor) if self.backend.is_complex(res.tensor) else res.tensor
        return self.backend.abs_square(res) if self.backend.is_complex(res) else res

    # ---------------------------------------------------------------- probabilities
    @staticmethod
    def _raw(res):
        if isinstance(res, TNTensor):
            res.scale_to(1.0)
            return res.tensor
        return res

    def calculate_full_probability(self, qctn, circuit_states_list, measure_input_list):
        """engine_siamese.py:561-581."""
        return self._raw(self.contract_with_compiled_strategy(qctn, circuit_states_list, measure_input_list, True))

    def _identity(self, measure_input_list):
        dim = next((m.shape[-1] for m in measure_input_list if m is not None), 1)
        ident = self.backend.eye(dim)
        if measure_input_list and measure_input_list[0].ndim == 3:
            ident = self.backend.expand(self.backend.unsqueeze(ident, 0), measure_input_list[0].shape[0], -1, -1)
        return ident

    def calculate_marginal_probability(self, qctn, circuit_states_list, measure_input_list,
                                       qubit_indices: List[int]):
        """engine_siamese.py:583-640: identity Mx on the unmeasured qubits."""
        if len(qubit_indices) != len(measure_input_list):
            raise ValueError("Length of qubit_indices must match length of measure_input_list")
        ident = self._identity(measure_input_list)
        full = [measure_input_list[qubit_indices.index(i)] if i in qubit_indices else ident
                for i in range(qctn.nqubits)]
        return self._raw(self.contract_with_compiled_strategy(qctn, circuit_states_list, full, True))

    def calculate_conditional_probability(self, qctn, circuit_states_list, measure_input_list,
                                          qubit_indices: List[int], target_indices: List[int]):
        """engine_siamese.py:642-734: (B, 2, K, K) stacking [joint, marginal] -> P(A|B)."""
        if len(qubit_indices) != len(measure_input_list):
            raise ValueError("Length of qubit_indices must match length of measure_input_list")
        ident = self._identity(measure_input_list)
        full = []
        for i in range(qctn.nqubits):
            if i in qubit_indices:
                m = measure_input_list[qubit_indices.index(i)]
                full.append(self.backend.stack([m, ident if i in target_indices else m], dim=1))
            else:
                full.append(self.backend.stack([ident, ident], dim=1))
        res = self._raw(self.contract_with_compiled_strategy(qctn, circuit_states_list, full, True))
        return res[:, 0] / (res[:, 1] + 1e-10)
