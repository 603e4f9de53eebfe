"""StrategyCompiler (mirror of tneq_qc/contractor/compiler.py:17-136).

Same registry semantics: class-level MODES / _strategies, register_strategy(strategy, modes),
compile() = compatible strategies of the mode -> min estimated cost -> compute_fn, and the same
errors (ValueError for a bad mode, RuntimeError "No compatible strategy found!").
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Tuple

from .base import ContractionStrategy


class StrategyCompiler:
    MODES = {
        "fast": ["einsum_default"],
        "balanced": ["mps_chain"],
        "full": ["mps_chain"],
    }
    _strategies: Dict[str, ContractionStrategy] = {}

    def __init__(self, mode: str = "fast"):
        if mode not in self.MODES:
            raise ValueError(f"Invalid mode '{mode}'. Must be one of {list(self.MODES.keys())}")
        self.mode = mode

    @classmethod
    def register_strategy(cls, strategy: ContractionStrategy, modes: List[str] = None):
        cls._strategies[strategy.name] = strategy
        if modes is not None:
            for mode in modes:
                if mode in cls.MODES and strategy.name not in cls.MODES[mode]:
                    cls.MODES[mode].append(strategy.name)

    @classmethod
    def get_registered_strategies(cls) -> Dict[str, ContractionStrategy]:
        return cls._strategies.copy()

    @property
    def strategies(self) -> Dict[str, ContractionStrategy]:
        return self._strategies

    def compile(self, qctn, shapes_info: Dict[str, Any], backend, **kwargs) -> Tuple[Callable, str, float]:
        cands = []
        for name in self.MODES[self.mode]:
            st = self._strategies.get(name)
            if st is None or not st.check_compatibility(qctn, shapes_info):
                continue
            cost = st.estimate_cost(qctn, shapes_info)
            fn = st.get_compute_function(qctn, shapes_info, backend, **kwargs)
            cands.append((cost, name, fn))
        if not cands:
            raise RuntimeError("No compatible strategy found!")
        cost, name, fn = min(cands, key=lambda c: c[0])
        return fn, name, cost

    def register_custom_strategy(self, strategy: ContractionStrategy, modes: List[str]):
        self.register_strategy(strategy, modes)
