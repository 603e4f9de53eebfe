"""ContractionStrategy ABC (mirror of tneq_qc/contractor/base.py:12-62)."""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Callable, Dict


class ContractionStrategy(ABC):
    """A way to turn (qctn, shapes_info) into compute_fn(cores_dict, circuit_states, measure_matrices)."""

    @abstractmethod
    def check_compatibility(self, qctn, shapes_info: Dict[str, Any]) -> bool:
        """Whether the network structure is supported."""

    @abstractmethod
    def get_compute_function(self, qctn, shapes_info: Dict[str, Any], backend) -> Callable:
        """Return compute_fn(cores_dict, circuit_states, measure_matrices[, right_cores_dict])."""

    @abstractmethod
    def estimate_cost(self, qctn, shapes_info: Dict[str, Any]) -> float:
        """Estimated cost; the compiler picks the cheapest compatible strategy."""

    @property
    @abstractmethod
    def name(self) -> str:
        """Registry name."""
