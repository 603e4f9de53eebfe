"""BackendFactory (mirror of tneq_qc/backends/backend_factory.py:16-100) with 'hip' registered.

create_backend(name, device=None, tensor_type=None, **kwargs) -> cls(device=..., tensor_type=..., **kwargs);
register_backend(name, cls) adds a backend; unknown names raise ValueError as in the reference.
The default backend is 'hip' (the reference defaults to 'jax' on 'gpu', backend_factory.py:79-89).
"""
from __future__ import annotations

from typing import Optional, Type

from .backend_hip import BackendHIP
from .backend_interface import ComputeBackend


class BackendFactory:
    _backends = {"hip": BackendHIP}
    _default_backend: Optional[str] = None
    _backend_instance: Optional[ComputeBackend] = None

    @classmethod
    def create_backend(cls, backend_name: str, device: Optional[str] = None,
                       tensor_type: Optional[str] = None, **kwargs) -> ComputeBackend:
        name = backend_name.lower()
        if name not in cls._backends:
            raise ValueError(f"Unknown backend: {name}. Available backends: {list(cls._backends.keys())}")
        return cls._backends[name](device=device, tensor_type=tensor_type, **kwargs)

    @classmethod
    def set_default_backend(cls, backend_name: str, device: Optional[str] = None,
                            tensor_type: Optional[str] = None, **kwargs):
        cls._default_backend = backend_name.lower()
        cls._backend_instance = cls.create_backend(backend_name, device=device,
                                                   tensor_type=tensor_type, **kwargs)

    @classmethod
    def get_default_backend(cls) -> ComputeBackend:
        if cls._backend_instance is None:
            cls.set_default_backend("hip")
        return cls._backend_instance

    @classmethod
    def register_backend(cls, name: str, backend_class: Type[ComputeBackend]):
        cls._backends[name.lower()] = backend_class
