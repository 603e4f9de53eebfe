"""Engine: the reference's legacy caller of the contraction path (tneq_qc/core/engine.py:19-343), on
the HIP backend.

It is the reference's only amplitude-vector API: ``contract_with_vector_inputs`` (engine.py:285-315)
builds the vector-inputs einsum (EinsumStrategy.build_with_vector_inputs_expression,
einsum_strategy.py:258-318), caches the contraction expression on the QCTN under the same
attribute the reference uses (``_contract_expr_vector_inputs_<shapes>``, set with setattr,
engine.py:303-308), and runs it through the backend (jit_compile + execute_expression).  The
expression is a HipContractExpression: the pairwise path runs as one native plan (permute / sweep /
MFMA GEMM kernels).  The other legacy entry points on the same path keep their caches too:
``contract_core_only`` (engine.py:228-252, ``_contract_expr_core_only``), ``contract_with_inputs``
(:254-283, ``_contract_expr_inputs_<shape>``) and ``contract_with_qctn`` (:317-343,
``_contract_expr_with_qctn``).  The reference's ``contract_with_self*`` (forced ``.cuda()`` calls,
engine.py:428-429) and its MPS-chain helpers are outside the hot path.
"""
from __future__ import annotations

from typing import List, Optional, Union

from ..backends.backend_factory import BackendFactory
from ..backends.backend_interface import ComputeBackend
from ..contractor import EinsumStrategy, StrategyCompiler


class Engine:
    def __init__(self, backend: Optional[Union[str, ComputeBackend]] = None, strategy_mode: str = "balanced"):
        # engine.py:29-51 (the reference creates a named backend on device "cuda")
        if backend is None:
            self.backend = BackendFactory.get_default_backend()
        elif isinstance(backend, str):
            self.backend = BackendFactory.create_backend(backend, device="cuda")
        else:
            self.backend = backend
        self.contractor = EinsumStrategy()
        self.strategy_compiler = StrategyCompiler(mode=strategy_mode)
        self.strategy_mode = strategy_mode

    def _run(self, qctn, cache_key: str, build, tensors):
        """Expression cached on the QCTN under `cache_key` (setattr, as the reference), then
        jit_compile + execute_expression on the backend."""
        if not hasattr(qctn, cache_key):
            einsum_eq, tensor_shapes = build()
            setattr(qctn, cache_key, self.contractor.create_contract_expression(einsum_eq, tensor_shapes))
        expr = getattr(qctn, cache_key)
        jit_fn = self.backend.jit_compile(expr)
        return self.backend.execute_expression(jit_fn, *tensors)

    def _cores(self, qctn):
        return [self.backend.convert_to_tensor(qctn.cores_weights[c]) for c in qctn.cores]

    def contract_core_only(self, qctn):
        """engine.py:228-252: the cores alone; output legs in core order."""
        return self._run(qctn, "_contract_expr_core_only",
                         lambda: self.contractor.build_core_only_expression(qctn), self._cores(qctn))

    def contract_with_inputs(self, qctn, inputs):
        """engine.py:254-283: one input tensor on the circuit-input legs."""
        inputs = self.backend.convert_to_tensor(inputs)
        key = f"_contract_expr_inputs_{inputs.shape}"
        return self._run(qctn, key, lambda: self.contractor.build_with_inputs_expression(qctn, inputs.shape),
                         [inputs] + self._cores(qctn))

    def contract_with_vector_inputs(self, qctn, inputs: List):
        """engine.py:285-315: psi = the circuit applied to the product state of `inputs` (one
        vector per circuit input, consumed in core / in-edge order); outputs open in core order."""
        inputs = [self.backend.convert_to_tensor(inp) for inp in inputs]
        inputs_shapes = [inp.shape for inp in inputs]
        key = f"_contract_expr_vector_inputs_{tuple(inputs_shapes)}"
        return self._run(qctn, key,
                         lambda: self.contractor.build_with_vector_inputs_expression(qctn, inputs_shapes),
                         inputs + self._cores(qctn))

    def contract_with_qctn(self, qctn, target_qctn):
        """engine.py:317-343: <target| qctn> style contraction of two QCTNs."""
        return self._run(qctn, "_contract_expr_with_qctn",
                         lambda: self.contractor.build_with_qctn_expression(qctn, target_qctn),
                         self._cores(qctn) + self._cores(target_qctn))
