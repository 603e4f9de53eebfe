"""EngineSiamese caller surface (mirror of tneq_qc/core/engine_siamese.py:20-734) on the HIP backend.

contract_with_compiled_strategy keeps the reference's contract: shapes_info -> per-QCTN cached
compute_fn from the StrategyCompiler (engine_siamese.py:261-317), execute, then the Born rule
(abs_square) for complex results and TNTensor.scale_to(1.0) (engine_siamese.py:319-349).
The probability helpers follow engine_siamese.py:561-734; unlike the reference they also accept
plain-tensor results (the reference calls .scale_to on a raw tensor there).
The training entry (contract_with_compiled_strategy_for_gradient, :351-554) differentiates through
the HIP expression's autograd; the measurement data (generate_data, :133-254) and the CDF block
of sample (:854-905) run on HIP kernels (ops.hermite_features / ops.inverse_cdf_sample).
"""
from __future__ import annotations

import math
from typing import Any, List, Optional, Union

import numpy as np

from .. import ops
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
    def __init__(self, backend: Optional[Union[str, ComputeBackend]] = None, strategy_mode: str = "balanced",
                 mx_K: int = 100):
        if backend is None:
            self.backend = BackendFactory.get_default_backend()
        elif isinstance(backend, str):
            self.backend = BackendFactory.create_backend(backend)
        else:
            self.backend = backend
        self.contractor = EinsumStrategy()
        self.strategy_compiler = StrategyCompiler(mode=strategy_mode)
        self.strategy_mode = strategy_mode
        self.mx_K = mx_K
        self.mx_weights = self._init_mx_weights(mx_K)

    # ---------------------------------------------------------------- measurement data
    def _init_mx_weights(self, k_max):
        """engine_siamese.py:59-80: w_k = exp(-(log(2 pi)/2 + lgamma(k+1))/2), k = 0..k_max, in
        float64 on the host (kept for the kernel's launch arguments) and as a backend tensor."""
        k = np.arange(k_max + 1, dtype=np.float64)
        log_factorial = np.array([math.lgamma(int(v) + 1) for v in k], dtype=np.float64)
        w = np.exp(-0.5 * (0.5 * math.log(2 * math.pi) + log_factorial)).astype(np.float64)
        self._mx_weights_np = w
        return self.backend.convert_to_tensor(w)

    def generate_data(self, x, K: int = None, ret_type: str = "tensor"):
        """engine_siamese.py:133-254: (Mx_list, phi_x) for a [B, D] batch x.  One HIP launch
        (ops.hermite_features) computes phi (B, D, K) and Mx (B, D, K, K); Mx_list[i] = Mx[:, i]
        (views, as the reference).  Complex backends compute in float64 from the real part of x,
        real backends in their own precision, exactly as the reference's two branches."""
        if K is None:
            K = self.mx_K
        x = self.backend.convert_to_tensor(x)
        if K > self.mx_K or K > self._mx_weights_np.shape[0]:
            self.mx_weights = self._init_mx_weights(K)
            self.mx_K = K
        phi, mx = ops.hermite_features(x, K, self._mx_weights_np, x.dtype)
        Mx_list = []
        for i in range(x.shape[1]):
            t = mx[:, i]
            if ret_type == "TNTensor":
                t = TNTensor(t)
                t.auto_scale()
            Mx_list.append(t)
        return Mx_list, phi

    def sample(self, qctn, circuit_states_list, num_samples, K, bounds=(-5, 5), grid_size=1000):
        """engine_siamese.py:740-915: sample one coordinate per qubit in turn by the numerical
        inverse CDF.  Qubit q's density over the grid comes from the contraction with the grid
        Mx on q, the Mx of the values already drawn on earlier qubits and the identity on later
        ones.  Same measurements and arithmetic as the reference; the measurements enter as
        stride-0 (S, G, K, K) views (batch symbols 'ab') instead of materialised (S*G, K, K)
        copies, and the CDF search runs in one HIP kernel per qubit."""
        b = self.backend
        torch = b.torch
        x_min, x_max = bounds
        S, G, n = int(num_samples), int(grid_size), qctn.nqubits
        grid_x = b.linspace(x_min, x_max, steps=G)
        ident = b.eye(K)
        persistent = [None] * n
        samples = b.zeros((S, n))
        Mx_grid = self.generate_data(b.unsqueeze(grid_x, 1), K=K)[0][0]       # (G, K, K)
        grid_r = (grid_x.real if grid_x.is_complex() else grid_x).contiguous()
        for q_idx in range(n):
            measures = []
            for i in range(n):
                if i == q_idx:
                    m = Mx_grid.unsqueeze(0).expand(S, G, K, K)
                elif i < q_idx:
                    m = persistent[i].unsqueeze(1).expand(S, G, K, K)
                else:
                    m = ident.expand(S, G, K, K)
                measures.append(m)
            res = self.contract_with_compiled_strategy(qctn, circuit_states_list, measures, measure_is_matrix=True)
            if isinstance(res, TNTensor):
                res = res.tensor
            density = b.abs_square(b.reshape(res, (S, G)))
            if density.is_complex():
                density = density.real
            u = b.rand((S, 1), dtype=torch.float32)
            y = ops.inverse_cdf_sample(density.contiguous(), grid_r.to(density.dtype), u)
            samples[:, q_idx] = y.to(samples.dtype)
            persistent[q_idx] = self.generate_data(b.unsqueeze(y, 1), K=K)[0][0]
        return samples

    # ---------------------------------------------------------------- training
    def contract_with_compiled_strategy_for_gradient(self, qctn, circuit_states_list, measure_input_list,
                                                     measure_is_matrix=True, right_qctn="symmetric"):
        """engine_siamese.py:351-554: (loss, grads) with loss = -mean(log(clamp(P, 1e-10)) +
        log_scale), P = |result|^2 for a complex result, gradients w.r.t. every core that requires
        grad (the QCTN's, then a right QCTN's).  Trainable TNTensor cores keep their scale
        (a constant); non-trainable TNTensor cores enter as their raw tensor, as the reference.
        Backward runs on the HIP engine: each operand's gradient is one more contraction
        (expression._HipContractFn)."""
        b = self.backend
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
        compute_fn = cached["compute_fn"]
        right_is_qctn = right_qctn is not None and not isinstance(right_qctn, str)

        def raw_of(c):
            return c.tensor if isinstance(c, TNTensor) else c

        def trainable(c):
            return bool(getattr(raw_of(c), "requires_grad", False))

        sources = [(qctn, name) for name in qctn.cores]
        if right_is_qctn:
            sources += [(right_qctn, name) for name in right_qctn.cores]
        raw, scales = [], []
        for owner, name in sources:
            c = owner.cores_weights[name]
            if trainable(c):
                raw.append(raw_of(c))
                scales.append(c.scale if isinstance(c, TNTensor) else 1.0)

        def loss_fn(*args):
            off = 0
            dicts = ({}, {})
            for owner, name in sources:
                c = owner.cores_weights[name]
                if trainable(c):
                    t = TNTensor(args[off], scales[off])
                    off += 1
                else:
                    t = raw_of(c)
                dicts[0 if owner is qctn else 1][name] = t
            result = compute_fn(dicts[0], circuit_states_list, measure_input_list, right_cores_dict=dicts[1])
            if isinstance(result, TNTensor):
                res, log_scale = result.tensor, result.log_scale
            else:
                res, log_scale = result, 0.0
            if b.is_complex(res):
                res = b.abs_square(res)
            target = b.ones(res.shape, dtype=res.dtype)
            res = b.clamp(res, min=1e-10)
            return -b.mean(target * (b.log(res) + b.detach(log_scale)))

        value_and_grad = b.compute_value_and_grad(loss_fn, argnums=list(range(len(raw))))
        return value_and_grad(*raw)

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
