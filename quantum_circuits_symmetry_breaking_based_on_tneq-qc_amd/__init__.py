"""tneq_qc_amd — MI355X-native contraction engine behind the tneq_qc plugin surface.

Import as ``import tneq_qc_amd`` (see the repo-root ``tneq_qc_amd.py`` alias).  Layout:
  csrc/         HIP kernels (permute, MFMA GEMM, small-operand apply) + C++ plan compiler/executor
  lib/          libtneqhip.so (built in-tree by __graft_entry__.build())
  _lib.py       ctypes binding of include/tneqhip.h (fails loudly if the .so is missing)
  ops.py        torch-tensor entry points over the C ABI
  einsum.py     equation parsing + path finders (greedy, linear sweep, cut tree) + slicing
  expression.py HipContractExpression: drop-in for opt_einsum.contract_expression(...)(*tensors)
  core/         QCTN / TNTensor host mirrors (graph bookkeeping of tneq_qc/core)
  backends/     ComputeBackend ABC, BackendFactory, BackendHIP ('hip')
  contractor/   ContractionStrategy ABC, StrategyCompiler, EinsumStrategy builders, HIP strategies
  distributed/  index-sliced multi-GPU contraction with an RCCL reduce of partial amplitudes
  circuits.py   brick-wall random-circuit generators used by the configs
"""
__version__ = "0.1.0"
