"""BackendInfo + ComputeBackend ABC (mirror of tneq_qc/backends/backend_interface.py:14-518).

Same abstract surface so a backend written against the reference's interface plugs in here
and vice versa; the 'hip' implementation is backends/backend_hip.py.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Optional

import numpy as np


class BackendInfo:
    """Backend configuration record (backend_interface.py:14-46)."""

    def __init__(self, backend_type: str, device: Optional[str] = None, dtype: Optional[str] = None,
                 **kwargs):
        self.backend_type = backend_type.lower()
        self.device = device
        self.dtype = dtype
        self.config = kwargs

    def __repr__(self):
        return (f"BackendInfo(backend_type='{self.backend_type}', device='{self.device}', "
                f"dtype='{self.dtype}', config={self.config})")

    __str__ = __repr__


class ComputeBackend(ABC):
    """Tensor-operation backend (backend_interface.py:48-518)."""

    def __init__(self, tensor_type: Optional[str] = None):
        self.backend_info: Optional[BackendInfo] = None
        self._tensor_type_name: Optional[str] = tensor_type

    # -- TNTensor helpers (backend_interface.py:68-100)
    @property
    def use_tn_tensor(self) -> bool:
        return self._tensor_type_name == "TNTensor"

    def wrap_tensor(self, tensor):
        if self.use_tn_tensor:
            from ..core.tn_tensor import TNTensor
            return tensor if isinstance(tensor, TNTensor) else TNTensor(tensor)
        return tensor

    def unwrap_tensor(self, tensor):
        from ..core.tn_tensor import TNTensor
        return tensor.tensor if isinstance(tensor, TNTensor) else tensor

    # -- abstract surface
    @abstractmethod
    def execute_expression(self, expression, *tensors): ...

    @abstractmethod
    def compute_value_and_grad(self, loss_fn, argnums): ...

    @abstractmethod
    def jit_compile(self, func): ...

    @abstractmethod
    def convert_to_tensor(self, array): ...

    @abstractmethod
    def optimizer_update(self, params, grads, state, method: str, hyperparams: dict): ...

    @abstractmethod
    def get_backend_name(self) -> str: ...

    def get_backend_info(self) -> BackendInfo:
        if self.backend_info is None:
            self.backend_info = BackendInfo(self.get_backend_name())
        return self.backend_info

    def set_backend_info(self, backend_info: BackendInfo):
        if backend_info.backend_type != self.get_backend_name():
            raise ValueError(f"BackendInfo type '{backend_info.backend_type}' does not match "
                             f"backend '{self.get_backend_name()}'")
        self.backend_info = backend_info

    @abstractmethod
    def init_random_core(self, shape): ...

    def get_tensor_type(self):
        if self.use_tn_tensor:
            from ..core.tn_tensor import TNTensor
            return TNTensor
        return self._get_raw_tensor_type()

    @abstractmethod
    def _get_raw_tensor_type(self): ...

    @abstractmethod
    def tensor_to_numpy(self, tensor) -> np.ndarray: ...

    @abstractmethod
    def set_random_seed(self, seed: int): ...

    @abstractmethod
    def reshape(self, tensor, shape): ...

    @abstractmethod
    def eye(self, n: int, dtype=None): ...

    @abstractmethod
    def zeros(self, shape, dtype=None): ...

    @abstractmethod
    def ones(self, shape, dtype=None): ...

    @abstractmethod
    def clone(self, tensor): ...

    @abstractmethod
    def unsqueeze(self, tensor, dim): ...

    @abstractmethod
    def expand(self, tensor, *sizes): ...

    @abstractmethod
    def clamp(self, tensor, min=None, max=None): ...

    @abstractmethod
    def diagonal(self, tensor, dim1=-2, dim2=-1): ...

    @abstractmethod
    def sum(self, tensor, dim=None, keepdim=False): ...

    @abstractmethod
    def multinomial(self, probs, num_samples): ...

    @abstractmethod
    def arange(self, *args, dtype=None): ...

    @abstractmethod
    def stack(self, tensors, dim=0): ...

    @abstractmethod
    def log(self, tensor): ...

    @abstractmethod
    def mean(self, tensor, dim=None, keepdim=False): ...

    @abstractmethod
    def squeeze(self, tensor, dim=None): ...

    @abstractmethod
    def einsum(self, equation: str, *operands): ...

    def is_complex(self, tensor) -> bool:
        return False

    def abs_square(self, tensor):
        return tensor
