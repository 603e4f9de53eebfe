"""Contractor: strategy ABC, compiler registry, einsum builders, HIP strategies
(mirror of tneq_qc/contractor/__init__.py:1-60: strategies are registered at import)."""
from .base import ContractionStrategy
from .compiler import StrategyCompiler
from .einsum_strategy import EinsumStrategy
from .hip_strategy import HipTreeStrategy


def _register_builtin_strategies():
    StrategyCompiler.register_strategy(EinsumStrategy(), modes=["fast"])
    StrategyCompiler.register_strategy(HipTreeStrategy(), modes=["balanced", "full"])


_register_builtin_strategies()

__all__ = ["ContractionStrategy", "EinsumStrategy", "HipTreeStrategy", "StrategyCompiler"]
